#!/usr/bin/env python3
"""Block-sparse attention forward (gfx950 flash kernel, SPARSE LUT) vs the dense flash forward and vs the
masked-SDPA path, at BigBird / Fixed layouts; one JSON line per config."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402
from deepspeedsyclsupport_amd.ops.sparse_attention import block_sparse as bs  # noqa: E402
from deepspeedsyclsupport_amd.ops.sparse_attention.sparsity_config import (BigBirdSparsityConfig,  # noqa: E402
                                                                            FixedSparsityConfig)


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    B, H, D = 2, 16, 128
    for L in (4096, 16384):
        for name, cfg in (("bigbird64", BigBirdSparsityConfig(num_heads=H, block=64)),
                          ("fixed64", FixedSparsityConfig(num_heads=H, block=64, num_local_blocks=4))):
            layout = cfg.make_layout(L)
            q, k, v = (torch.randn(B, H, L, D, device="cuda").bfloat16() for _ in range(3))
            tiles, ntiles, lay, qorder = bs.build_lut(layout, cfg.block, L, q.device)
            density = ntiles.float().mean().item() / (L // 64)
            t_sparse = timeit(lambda: hip_ops().flash_fwd_sparse(q, k, v, D**-0.5, tiles, ntiles, qorder, lay,
                                                                 cfg.block, False))
            t_dense = timeit(lambda: hip_ops().flash_fwd(q, k, v, False, D**-0.5, False))
            bias = bs.token_bias(layout, cfg.block, L, H, torch.bfloat16, q.device)
            t_sdpa = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=bias))
            # masks applied in-kernel: BERT key padding (per key), attention mask + rpe (per row and key), fwd + bwd
            qg, kg, vg = (t.clone().requires_grad_(True) for t in (q, k, v))
            kpm = torch.zeros(B, L, device="cuda")
            kpm[:, L - L // 8:] = -10000.0
            am = torch.zeros(L, L, device="cuda")
            rpe = torch.randn(H, L, L, device="cuda") if L <= 4096 else None

            def fb(**kw):
                o = bs.block_sparse_attention(qg, kg, vg, layout, cfg.block, **kw)
                o.backward(o)
                qg.grad = kg.grad = vg.grad = None

            t_fb = timeit(lambda: fb())
            t_fb_kpm = timeit(lambda: fb(key_padding_mask=kpm))
            t_fb_all = timeit(lambda: fb(key_padding_mask=kpm, attn_mask=am, attn_mask_mode="add", rpe=rpe))
            t_f_kpm = timeit(lambda: bs.block_sparse_attention(q, k, v, layout, cfg.block, key_padding_mask=kpm))
            extra = {"fwd_bwd_ms": round(t_fb, 3), "fwd_bwd_padding_mask_ms": round(t_fb_kpm, 3),
                     "fwd_bwd_padding_attn_mask_rpe_ms": round(t_fb_all, 3), "rpe": rpe is not None,
                     "fwd_padding_mask_ms": round(t_f_kpm, 3)}
            del rpe, am
            print(json.dumps({"layout": name, **extra, "B": B, "H": H, "L": L, "D": D, "tile_density": round(density, 3),
                              "sparse_fwd_ms": round(t_sparse, 3), "dense_flash_fwd_ms": round(t_dense, 3),
                              "masked_sdpa_fwd_ms": round(t_sdpa, 3),
                              "speedup_vs_masked_sdpa": round(t_sdpa / t_sparse, 2)}), flush=True)
            del bias


if __name__ == "__main__":
    main()
