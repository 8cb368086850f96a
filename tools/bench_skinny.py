#!/usr/bin/env python3
"""Decode GEMM micro-benchmark: VALU skinny vs MFMA skinny vs hipBLASLt (F.linear) on Llama-2-7B shapes.
Prints one JSON line per (shape, M, path) with time and effective weight-stream bandwidth."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    ops = hip_ops()
    dev = "cuda"
    shapes = {"qkv": (12288, 4096, False, 1), "o": (4096, 4096, False, 0), "gate_up": (22016, 4096, True, 1),
              "down": (4096, 11008, False, 0), "lm_head": (32000, 4096, False, 1)}
    nw = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    for name, (N, K, gated, in_mode) in shapes.items():
        # rotate through > 1 GB of weight copies so every call streams from HBM (MI355X has a 256 MB MALL)
        ncopy = max(2, int(1.2e9 // (N * K * 2)) + 1)
        Ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        it = [0]

        def W_next():
            it[0] = (it[0] + 1) % ncopy
            return Ws[it[0]]
        for M in (1, 2, 4, 8, 16):
            x = torch.randn(M, K, device=dev).bfloat16()
            r = torch.randn(M, K, device=dev).bfloat16()
            res = torch.empty_like(x)
            for path in ("valu", "mfma", "auto", "blas"):
                if path == "valu" and M > 8:
                    continue
                if path == "blas":
                    fn = lambda: torch.nn.functional.linear(x, W_next())  # noqa: E731
                else:
                    ops.skinny_set_path({"valu": 1, "mfma": 2, "auto": 0}[path])
                    fn = lambda: ops.skinny_gemm(x, W_next(), None, None, in_mode, gated, 0, r if in_mode else None,  # noqa
                                                 nw if in_mode else None, 1e-5, res if in_mode else None)
                us = timeit(fn)
                print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "path": path, "us": round(us, 2),
                                  "TBps": round(N * K * 2 / us / 1e6, 2)}), flush=True)
    ops.skinny_set_path(0)


if __name__ == "__main__":
    main()
