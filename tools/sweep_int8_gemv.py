#!/usr/bin/env python3
"""Interleaved sweep of the int8 MFMA GEMV variants in ONE process (box-to-box variance is large, so variants are
compared side by side): `python tools/sweep_int8_gemv.py cfg:wpc[:dbg] ...`."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.int8_gemv import preshuffle  # noqa: E402
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


variants = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(0, 8)]
for N, K in ((57344, 14336), (14336, 57344), (22016, 4096)):
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    qt = quantize(w, group_size=64, bits=8)
    del w
    qsh, ssh = preshuffle(qt.data.view(N, K), qt.scales, 64)
    nbytes = N * K * (1 + 4 / 64)
    for M in (1, 8, 16):
        x = torch.randn(M, K, device="cuda").bfloat16()
        row = {"N": N, "K": K, "M": M}
        if M <= 8:
            row["valu"] = round(nbytes / timeit(lambda: hip_ops().skinny_i8(x, qt.data, qt.scales, None, N, 64)) / 1e12, 2)
        for rep in range(2):
            for v in variants:
                hip_ops().skinny_i8_tune(v[0], v[1], v[2] if len(v) > 2 else 0)
                t = timeit(lambda: hip_ops().skinny_i8_sh(x, qsh, ssh, None, N, 64))
                key = ":".join(map(str, v))
                row[key] = max(row.get(key, 0), round(nbytes / t / 1e12, 2))
        print(json.dumps(row), flush=True)
