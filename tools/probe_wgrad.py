#!/usr/bin/env python3
"""Weight-gradient GEMM formulations for the Llama-2-7B step (T = 32768 tokens), each tuned with PyTorch TunableOp:
  A: dW = dY^T . X            (what nn.Linear's backward issues)
  B: dW^T = X^T . dY, then one transpose copy into [out, in]
  C: A with fp32 output (out_dtype)
  D: K-major operands: dY^T and X^T materialised contiguous ([out, T], [in, T]) by a transpose copy, then a TN GEMM
     (the layout the forward GEMMs run at ~2 PF/s)
Prints one JSON line per shape with ms and PF/s."""
import json
import os
import sys
import threading
import time

import torch

T = int(os.environ.get("T", "32768"))
SHAPES = [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096)]


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(20)
    tun.set_max_tuning_iterations(10)
    tun.set_filename(os.path.join("gpurun_out", "probe_wgrad_tunable.csv"), False)
    t0 = time.time()

    def hb():
        while True:
            time.sleep(20)
            print(f"# alive {time.time() - t0:.0f}s", flush=True)

    threading.Thread(target=hb, daemon=True).start()
    for out_f, in_f in SHAPES:
        dY = torch.randn(T, out_f, device="cuda", dtype=torch.bfloat16)
        X = torch.randn(T, in_f, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * out_f * in_f
        row = {"out": out_f, "in": in_f, "T": T}
        row["A_ms"] = timed(lambda: torch.mm(dY.t(), X))
        Bt = None
        dYt, Xt = dY.t().contiguous(), X.t().contiguous()
        row["D_gemm_ms"] = timed(lambda: torch.mm(dYt, Xt.t()))
        row["D_transposes_ms"] = timed(lambda: (dY.t().contiguous(), X.t().contiguous()))
        row["D_pflops"] = round(fl / row["D_gemm_ms"] / 1e12, 3)
        del dYt, Xt
        for k in ("A_ms", ):
            row[k.replace("_ms", "_pflops")] = round(fl / row[k] / 1e12, 3)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
        del dY, X, Bt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
