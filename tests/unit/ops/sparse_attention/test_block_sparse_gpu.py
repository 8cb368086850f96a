"""Block-sparse flash kernel vs a dense fp32 reference with the layout as an additive mask (reference
`tests/unit/ops/sparse_attention/test_sparse_attention.py`: sparse softmax / matmul vs dense on the same layout)."""
import pytest
import torch

from deepspeedsyclsupport_amd.ops.sparse_attention import block_sparse as bs
from deepspeedsyclsupport_amd.ops.sparse_attention.sparsity_config import (BigBirdSparsityConfig,
                                                                            BSLongformerSparsityConfig,
                                                                            FixedSparsityConfig,
                                                                            VariableSparsityConfig)

pytestmark = pytest.mark.gpu


def _dense_ref(q, k, v, layout, blk, scale):
    B, H, L, D = q.shape
    bias = bs.token_bias(layout, blk, L, H, torch.float32, q.device)
    s = (q.float() @ k.float().transpose(-1, -2)) * scale + bias
    return torch.softmax(s, -1) @ v.float()


CFGS = [
    ("fixed16", lambda H: FixedSparsityConfig(num_heads=H, block=16, num_local_blocks=4)),
    ("fixed64_uni", lambda H: FixedSparsityConfig(num_heads=H, block=64, num_local_blocks=2,
                                                  attention="unidirectional")),
    ("bigbird32", lambda H: BigBirdSparsityConfig(num_heads=H, block=32)),
    ("longformer128", lambda H: BSLongformerSparsityConfig(num_heads=H, block=128)),
    ("variable_perhead", lambda H: VariableSparsityConfig(num_heads=H, block=32, different_layout_per_head=True)),
]


@pytest.mark.parametrize("name,mk", CFGS, ids=[c[0] for c in CFGS])
@pytest.mark.parametrize("D", [64, 128])
def test_block_sparse_fwd_bwd(name, mk, D):
    torch.manual_seed(0)
    B, H, L = 2, 4, 1024
    cfg = mk(H)
    layout = cfg.make_layout(L)
    q, k, v = (torch.randn(B, H, L, D, device="cuda").bfloat16().requires_grad_(True) for _ in range(3))
    scale = D**-0.5
    assert bs.native_ok(q, k, v, cfg.block)
    o = bs.block_sparse_attention(q, k, v, layout, cfg.block)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _dense_ref(qr, kr, vr, layout, cfg.block, scale)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(ref)
    o.backward(do.bfloat16())
    ref.backward(do)
    for a, b, n in ((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")):
        err = (a.float() - b).abs().max().item()
        assert err < 5e-2 * max(1.0, b.abs().max().item()), f"{name} D={D} {n} err {err}"


def test_sparse_self_attention_module_uses_kernel():
    from deepspeedsyclsupport_amd.ops.sparse_attention.sparse_self_attention import SparseSelfAttention
    torch.manual_seed(1)
    H, L, D = 4, 2048, 64
    cfg = BigBirdSparsityConfig(num_heads=H, block=64)
    attn = SparseSelfAttention(cfg)
    q, k, v = (torch.randn(1, H, L, D, device="cuda").bfloat16() for _ in range(3))
    o = attn(q, k, v)
    ref = _dense_ref(q, k, v, attn.get_layout(L), 64, D**-0.5)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    tiles, ntiles, _, _ = bs.build_lut(attn.get_layout(L), 64, L, q.device)
    assert ntiles.float().mean().item() < 0.5 * (L // 64)  # the kernel really skips most key tiles


def test_block_sparse_bwd_long_sequence_memory():
    """16k tokens x 16 heads: a dense [B,H,L,L] bias would be 8 GB in bf16; the sparse backward must stay within a
    small multiple of the activations and match a chunked reference on a slice of rows."""
    torch.manual_seed(2)
    B, H, L, D = 1, 16, 16384, 64
    cfg = BigBirdSparsityConfig(num_heads=H, block=64)
    layout = cfg.make_layout(L)
    q, k, v = (torch.randn(B, H, L, D, device="cuda").bfloat16().requires_grad_(True) for _ in range(3))
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    o = bs.block_sparse_attention(q, k, v, layout, 64)
    do = torch.randn_like(o)
    o.backward(do)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    assert peak < 2 * 1024**3, peak  # activations + fp32 dq accumulator; no L x L tensor
    # reference on the first 128 query rows of head 0: dv of keys gets contributions from all rows, so check dq
    tok = layout[0].bool().repeat_interleave(64, 0).repeat_interleave(64, 1)[:128].cuda()
    qs = q[0, 0, :128].detach().float()
    s = (qs @ k[0, 0].detach().float().T) * D**-0.5
    s = s.masked_fill(~tok, float("-inf"))
    p = torch.softmax(s, -1)
    dp = do[0, 0, :128].float() @ v[0, 0].detach().float().T
    ds = p * (dp - (p * dp).sum(-1, keepdim=True))
    ref_dq = (ds @ k[0, 0].detach().float()) * D**-0.5
    torch.testing.assert_close(q.grad[0, 0, :128].float(), ref_dq, rtol=5e-2, atol=5e-2)
