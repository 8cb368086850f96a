#!/usr/bin/env python3
"""MoE block microbenchmark on one MI355X: the sync-free gfx950 path (top-k gating -> scatter -> grouped MFMA GEMM ->
SwiGLU -> grouped GEMM -> weighted gather, `ops/moe_ops.py`) vs the per-expert PyTorch loop (bincount().tolist() host
sync + one hipBLASLt GEMM pair per expert). Mixtral-8x7B layer shapes (H 4096, I 14336, E 8, top-2), bf16.
Prints one JSON line per token count."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops import moe_ops  # noqa: E402
from deepspeedsyclsupport_amd.ops.transformer import functional as DF  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    H, I, E, k = 4096, 14336, 8, 2
    torch.manual_seed(0)
    dev = "cuda"
    rw = (torch.randn(E, H, device=dev) / H**0.5).bfloat16()
    w1 = (torch.randn(E, 2 * I, H, device=dev) / H**0.5).bfloat16()
    w2 = (torch.randn(E, H, I, device=dev) / I**0.5).bfloat16()
    act = lambda h: DF.gated_activation(h, "silu")  # noqa: E731
    for T in [int(t) for t in os.environ.get("MOE_TOKENS", "16,256,2048,8192").split(",")]:
        x = torch.randn(T, H, device=dev).bfloat16()
        flops = 2 * T * k * (H * 2 * I + I * H)
        t_native = timeit(lambda: moe_ops.moe_block(x, rw, w1, w2, k, act, True))
        t_loop = timeit(lambda: moe_ops.moe_block_reference(x, rw, w1, w2, k, act, True))
        # grouped GEMM alone (first projection) for a kernel-level TF/s
        sc, ex, sl, cnt = moe_ops.topk_gating(F.linear(x, rw), k, True)
        xs, rows, _ = moe_ops.moe_scatter(x, ex, sl, cnt)
        t_gg = timeit(lambda: moe_ops.grouped_gemm(xs, w1, cnt))
        print(json.dumps({"tokens": T, "H": H, "I": I, "E": E, "top_k": k,
                          "native_ms": round(t_native, 3), "torch_loop_ms": round(t_loop, 3),
                          "speedup": round(t_loop / t_native, 2),
                          "native_block_tflops": round(flops / t_native / 1e9, 1),
                          "grouped_gemm_fc1_ms": round(t_gg, 3),
                          "grouped_gemm_fc1_tflops": round(2 * T * k * H * 2 * I / t_gg / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
