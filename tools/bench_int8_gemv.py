#!/usr/bin/env python3
"""Int8 weight-only skinny GEMM paths (VALU stream vs MFMA) at BLOOM-176B / Llama shapes: effective weight TB/s."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402
from deepspeedsyclsupport_amd.ops.quantizer import quantize  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


for N, K in ((57344, 14336), (14336, 57344), (43008, 14336), (11008 * 2, 4096)):
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    qt = quantize(w, group_size=64, bits=8)
    del w
    for M in (1, 2, 4, 8, 16):
        x = torch.randn(M, K, device="cuda").bfloat16()
        row = {"N": N, "K": K, "M": M}
        for path, name in ((1, "valu"), (2, "mfma")):
            if path == 1 and M > 8:
                continue
            t = timeit(lambda: hip_ops().skinny_i8(x, qt.data, qt.scales, None, N, 64, path))
            row[f"{name}_us"] = round(t * 1e6, 1)
            row[f"{name}_tb_s"] = round((N * K * (1 + 4 / 64)) / t / 1e12, 2)
        print(json.dumps(row), flush=True)
