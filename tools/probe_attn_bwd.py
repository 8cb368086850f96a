"""Probe: can the SDPA memory-efficient backward (aten._scaled_dot_product_efficient_attention_backward) consume an
(out, logsumexp) pair produced by another forward? Prints the forward's LSE shape/dtype and the max grad error when
the backward is fed a torch-computed fp32 LSE [B,H,S] instead of its own."""
import math
import torch
import torch.nn.functional as F

torch.manual_seed(0)
B, H, S, D = 2, 4, 1024, 128
dev = "cuda"
q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16) for _ in range(3))
do = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16)
scale = 1.0 / math.sqrt(D)
for causal in (True, False):
    out, lse, seed, off = torch.ops.aten._scaled_dot_product_efficient_attention(q, k, v, None, True, 0.0, causal,
                                                                                  scale=scale)
    print("causal", causal, "out", tuple(out.shape), "lse", tuple(lse.shape), lse.dtype, "seed", seed, off)
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, S, device=dev, dtype=torch.bool).triu(1), float("-inf"))
    lse_ref = torch.logsumexp(s, dim=-1)
    print("  lse vs ref max err", (lse[..., :S].float() - lse_ref).abs().max().item())
    g_own = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
        do, q, k, v, None, out, lse, seed, off, 0.0, [True, True, True, False], causal, scale=scale)
    lse_mine = torch.zeros_like(lse)
    lse_mine[..., :S] = lse_ref
    g_mine = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
        do, q, k, v, None, out, lse_mine.contiguous(), seed, off, 0.0, [True, True, True, False], causal, scale=scale)
    for n, a, b in zip("qkv", g_own[:3], g_mine[:3]):
        print(f"  d{n}: max|own-mine| {(a.float() - b.float()).abs().max().item():.3e}  max|own| {a.float().abs().max().item():.3e}")
    z = torch.zeros((), dtype=torch.int64, device=dev)
    try:
        g_z = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
            do, q, k, v, None, out, lse_mine.contiguous(), z, z, 0.0, [True, True, True, False], causal, scale=scale)
        print("  zero seed/offset ok, dq diff", (g_z[0].float() - g_own[0].float()).abs().max().item())
    except Exception as e:
        print("  zero seed/offset failed:", e)
