#!/usr/bin/env python3
"""Int4 weight-only skinny GEMM (fused-dequant MFMA stream over the packed weight) at Llama-7B / 70B / BLOOM shapes:
packed-byte TB/s and the bf16-equivalent rate, next to the int8 stream on the same shapes.

    python tools/bench_int4_gemv.py [quick]
Bytes counted: the HBM stream the op must read (packed int4 weights + fp32 group scales).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.int4_gemv import Int4Weight  # noqa: E402
from deepspeedsyclsupport_amd.ops.int8_gemv import Int8Weight  # noqa: E402
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


quick = "quick" in sys.argv[1:]
shapes = ((12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (57344, 14336), (14336, 57344), (28672, 8192))
for N, K in shapes[:4] if quick else shapes:
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    for gs in (128, 64):
        w4 = Int4Weight(w, gs)
        w8 = Int8Weight(w, gs) if gs == 64 else None
        for M in (1, 4, 8, 16):
            x = torch.randn(M, K, device="cuda").bfloat16()
            row = {"N": N, "K": K, "M": M, "gs": gs}
            for P, wpc, rounds in ((0, 0, 0), (3, 8, 2), (2, 8, 2), (2, 12, 1), (3, 8, 1), (2, 16, 1), (2, 12, 4)):
                hip_ops().skinny_i4_tune(P, wpc, rounds)
                # main kernel only (sums left in the workspace, re-zeroed by a plain finalize outside the timing)
                t = timeit(lambda: hip_ops().skinny_i4(x, w4.q4, w4.s4, None, N, gs))
                tag = "i4" if P == 0 else f"i4_p{P}w{wpc}r{rounds}"
                row[f"{tag}_us"] = round(t * 1e6, 1)
                row[f"{tag}_packed_tb_s"] = round(w4.nbytes() / t / 1e12, 2)
                if P == 0:
                    row["i4_bf16_equiv_tb_s"] = round(N * K * 2 / t / 1e12, 2)
            hip_ops().skinny_i4_tune(0, 0, 0)
            if w8 is not None:
                t = timeit(lambda: w8.linear(x))
                row["i8_us"] = round(t * 1e6, 1)
                row["i8_tb_s"] = round(w8.nbytes() / t / 1e12, 2)
            print(json.dumps(row), flush=True)
    del w
