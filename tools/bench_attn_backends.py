#!/usr/bin/env python3
"""SDPA backend study on the 7B training attention shape (B=8, H=32, S=4096, D=128, causal, bf16)."""
import json

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel


def bench(fn, it=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


B, H, S, D = 8, 32, 4096, 128
q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
g = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
fl_f = 4 * B * H * S * S * D / 2
libs = ["default"]
if hasattr(torch.backends.cuda, "preferred_rocm_fa_library"):
    libs = ["aotriton", "ck"]
for lib in libs:
    if lib != "default":
        try:
            torch.backends.cuda.preferred_rocm_fa_library(lib)
        except Exception as ex:
            print(json.dumps({"lib": lib, "error": str(ex)[:200]}))
            continue
    for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION):
        try:
            with sdpa_kernel(be):
                tf = bench(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True))

                def fb():
                    o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
                    torch.autograd.grad(o, (q, k, v), g)

                tfb = bench(fb)
            print(json.dumps({"lib": lib, "backend": be.name, "fwd_ms": round(tf, 3),
                              "fwd_TF": round(fl_f / tf / 1e9), "fwd_bwd_ms": round(tfb, 3),
                              "fwd_bwd_TF": round(3.5 * fl_f / tfb / 1e9)}), flush=True)
        except Exception as ex:
            print(json.dumps({"lib": lib, "backend": be.name, "error": str(ex)[:200]}), flush=True)
