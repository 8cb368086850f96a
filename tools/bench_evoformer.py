#!/usr/bin/env python3
"""DS4Sci Evoformer attention on one MI355X, the reference benchmark's shapes
(`tests/benchmarks/DS4Sci_EvoformerAttention_bench.py`: N=256 MSA rows, S=256, H=4, D=32, bf16, both biases,
bias2 with grad). Compares the fused kernel against the reference's own eager baseline (explicit softmax over the
materialised [B, N, H, S, S] logits) and against torch SDPA with the summed bias. One JSON line per batch."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def eager(Q, K, V, b1, b2, scale):
    q, k, v = (t.transpose(-2, -3) for t in (Q, K, V))
    a = torch.matmul(q * scale, k.transpose(-1, -2)) + b1 + b2
    return torch.matmul(torch.softmax(a.float(), -1).to(q.dtype), v).transpose(-2, -3)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(iters):
        st.record()
        fn()
        en.record()
        torch.cuda.synchronize()
        res.append(st.elapsed_time(en))
    res.sort()
    return res[len(res) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,4,16")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--D", type=int, default=32)
    args = ap.parse_args()
    from deepspeedsyclsupport_amd.ops import deepspeed4science as E
    N, S, H, D = args.N, args.S, args.H, args.D
    for B in [int(b) for b in args.batches.split(",")]:
        mk = lambda *s: torch.randn(*s, device="cuda", dtype=torch.bfloat16)  # noqa: E731
        Q, K, V = (mk(B, N, S, H, D).requires_grad_(True) for _ in range(3))
        b1 = mk(B, N, 1, 1, S)
        b2 = mk(B, 1, H, S, S).requires_grad_(True)
        do = torch.rand(B, N, S, H, D, device="cuda", dtype=torch.bfloat16)
        row = {"batch": B, "N": N, "S": S, "H": H, "D": D}
        paths = {"fused": lambda: E.DS4Sci_EvoformerAttention(Q, K, V, [b1, b2]),
                 "sdpa": lambda: E._sdpa_path(Q, K, V, [b1, b2]),
                 "eager": lambda: eager(Q, K, V, b1, b2, D**-0.5)}
        for name, fn in paths.items():
            try:
                out = fn()
                row[f"{name}_fwd_ms"] = round(timed(lambda: fn(), args.iters), 3)
                row[f"{name}_bwd_ms"] = round(timed(lambda: torch.autograd.grad(fn(), (Q, K, V, b2), do),
                                                    args.iters) - row[f"{name}_fwd_ms"], 3)
                del out
            except torch.OutOfMemoryError:
                row[f"{name}_fwd_ms"] = "oom"
            torch.cuda.empty_cache()
        fl = 4 * B * N * H * S * S * D
        row["fused_fwd_tflops"] = round(fl / row["fused_fwd_ms"] / 1e9, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
