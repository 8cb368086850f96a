#!/usr/bin/env python3
"""Weight-gradient GEMM layout study on Llama-2-7B shapes (MB=8 x 4096 tokens): which operand layout does
hipBLASLt run fastest for dW = dY^T X ?"""
import json

import torch


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


T = 32768
for name, (N, K) in {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
                     "lm_head": (32000, 4096)}.items():
    dY = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    X = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * N * K
    res = {}
    res["nt_dYt_X"] = t(lambda: dY.t() @ X)
    res["copyT_then_mm"] = t(lambda: dY.t().contiguous() @ X)
    res["XtdY_then_T"] = t(lambda: (X.t() @ dY).t().contiguous())
    res["XtdY_noT"] = t(lambda: X.t() @ dY)
    res["dgrad_dY_W"] = t(lambda: dY @ torch.empty(N, K, device="cuda", dtype=torch.bfloat16))
    print(json.dumps({"shape": name, "N": N, "K": K, **{k: f"{v:.3f}ms {fl / v / 1e9:.0f}TF" for k, v in res.items()}}),
          flush=True)
