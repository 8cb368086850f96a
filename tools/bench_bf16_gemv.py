#!/usr/bin/env python3
"""bf16 decode GEMV: the pre-shuffled MFMA stream (cfg / waves-per-CU variants) next to the row-major kernels, at
Llama-2-7B and BLOOM-176B projection shapes. One JSON line per (shape, rows, variant): time and TB/s of weight bytes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, reps=5):
    for _ in range(3):
        fn()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best * 1e3  # us


def main():
    from deepspeedsyclsupport_amd.ops.bf16_gemv import Bf16Weight
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    ops = hip_ops()
    shapes = [("7b_qkv", 12288, 4096), ("7b_o", 4096, 4096), ("7b_gate_up", 22016, 4096), ("7b_down", 4096, 11008),
              ("bloom_qkv", 43008, 14336), ("bloom_fc2", 14336, 57344)]
    variants = [(c, w) for c in (1, 2, 3, 4) for w in (8, 12, 16)]
    for name, N, K in shapes:
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        bw = Bf16Weight(w)
        gb = N * K * 2 / 1e12
        for M in [int(m) for m in os.environ.get("ROWS", "1,8,16").split(",")]:
            x = torch.randn(M, K, device="cuda").bfloat16()
            t = timeit(lambda: ops.skinny_gemm(x, w, None, None, 0, False, 0, None, None, 0.0, None))
            print(json.dumps({"shape": name, "N": N, "K": K, "rows": M, "kernel": "row_major", "us": round(t, 2),
                              "tb_s": round(gb / (t * 1e-6), 2)}), flush=True)
            best = None
            for cfg, wpc in variants:
                ops.skinny_b16_tune(cfg, wpc)
                t = timeit(lambda: bw.linear(x))
                rec = {"shape": name, "N": N, "K": K, "rows": M, "kernel": f"shuffled cfg{cfg} wpc{wpc}",
                       "us": round(t, 2), "tb_s": round(gb / (t * 1e-6), 2)}
                if os.environ.get("ALL"):
                    print(json.dumps(rec), flush=True)
                if best is None or t < best["us"]:
                    best = rec
            ops.skinny_b16_tune(0, 0)
            t = timeit(lambda: bw.linear(x))
            print(json.dumps({**best, "best": True}), flush=True)
            print(json.dumps({"shape": name, "N": N, "K": K, "rows": M, "kernel": "shuffled default", "us": round(t, 2),
                              "tb_s": round(gb / (t * 1e-6), 2)}), flush=True)
        del w, bw


if __name__ == "__main__":
    main()
