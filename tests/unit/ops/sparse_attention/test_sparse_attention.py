"""Sparse attention layouts and block-sparse attention vs a dense reference (reference
`tests/unit/ops/sparse_attention/test_sparse_attention.py`), and Evoformer attention vs an explicit softmax."""
import math

import pytest
import torch

from deepspeedsyclsupport_amd.ops import sparse_attention as sa


def test_fixed_layout_structure():
    cfg = sa.FixedSparsityConfig(num_heads=2, block=4, num_local_blocks=4, num_global_blocks=1)
    lay = cfg.make_layout(64)            # 16 blocks
    assert lay.shape == (2, 16, 16)
    assert lay[0, :4, :4].all()          # local window
    assert lay[0, :, 3].all()            # last block of each window is global (vertical, bidirectional)
    assert torch.equal(lay[0], lay[1])   # single layout propagated
    uni = sa.FixedSparsityConfig(num_heads=1, block=4, attention="unidirectional").make_layout(32)
    assert torch.equal(uni[0], torch.tril(uni[0]))


@pytest.mark.parametrize("cfg", [
    sa.DenseSparsityConfig(num_heads=2, block=8),
    sa.FixedSparsityConfig(num_heads=2, block=8, num_local_blocks=2),
    sa.BigBirdSparsityConfig(num_heads=2, block=8, num_random_blocks=1, num_sliding_window_blocks=3),
    sa.BSLongformerSparsityConfig(num_heads=2, block=8),
    sa.VariableSparsityConfig(num_heads=2, block=8, local_window_blocks=[2, 4]),
    sa.LocalSlidingWindowSparsityConfig(num_heads=2, block=8),
])
def test_sparse_attention_matches_dense_masked(cfg):
    torch.manual_seed(0)
    B, H, L, D = 2, 2, 64, 16
    q, k, v = (torch.randn(B, H, L, D) for _ in range(3))
    attn = sa.SparseSelfAttention(cfg)
    out = attn(q, k, v)
    lay = attn.get_layout(L) if isinstance(cfg, sa.DenseSparsityConfig) else attn.sparsity_config.make_layout(L)
    lay = attn._block_mask(L, q.device)[None]  # the cached mask actually used
    s = q @ k.transpose(-1, -2) / math.sqrt(D) + lay
    ref = torch.softmax(s, -1) @ v
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


def test_evoformer_attention_grads():
    from deepspeedsyclsupport_amd.ops.deepspeed4science import DS4Sci_EvoformerAttention
    torch.manual_seed(0)
    B, N, S, H, D = 1, 3, 8, 2, 16
    Q, K, V = (torch.randn(B, N, S, H, D, requires_grad=True) for _ in range(3))
    b1 = torch.randn(B, N, 1, 1, S, requires_grad=True)
    b2 = torch.randn(B, 1, H, S, S, requires_grad=True)
    out = DS4Sci_EvoformerAttention(Q, K, V, [b1, b2])
    q, k, v = (t.permute(0, 1, 3, 2, 4) for t in (Q, K, V))
    ref = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D) + b1 + b2, -1) @ v
    ref = ref.permute(0, 1, 3, 2, 4)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, (Q, b1, b2), g)
    gb = torch.autograd.grad(ref, (Q, b1, b2), g)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
