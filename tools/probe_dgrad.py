#!/usr/bin/env python3
"""Data-gradient GEMM layouts for the Llama-2-7B step (T = 32768): dX = dY . W with W row-major [out, in] (B operand
MN-major, what nn.Linear issues) vs dY . (W^T)^T with a K-major copy W^T [in, out]. TunableOp-tuned; one JSON line
per shape."""
import json
import os
import threading
import time

import torch

T = 32768
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
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(20)
    tun.set_max_tuning_iterations(10)
    tun.set_filename(os.path.join("gpurun_out", "probe_dgrad_tunable.csv"), False)
    t0 = time.time()

    def hb():
        while True:
            time.sleep(20)
            print(f"# alive {time.time() - t0:.0f}s", flush=True)

    threading.Thread(target=hb, daemon=True).start()
    for out_f, in_f in SHAPES:
        dY = torch.randn(T, out_f, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(out_f, in_f, device="cuda", dtype=torch.bfloat16)
        Wt = hip_ops().transpose16(W)
        fl = 2.0 * T * out_f * in_f
        row = {"out": out_f, "in": in_f, "T": T}
        row["nn_ms"] = timed(lambda: torch.mm(dY, W))
        row["kmajor_ms"] = timed(lambda: torch.mm(dY, Wt.t()))
        row["w_transpose_ms"] = timed(lambda: hip_ops().transpose16(W))
        row["nn_pflops"] = fl / row["nn_ms"] / 1e12
        row["kmajor_pflops"] = fl / row["kmajor_ms"] / 1e12
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
        del dY, W, Wt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
