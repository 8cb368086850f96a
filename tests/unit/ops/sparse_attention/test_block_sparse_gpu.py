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


def _masked_ref(q, k, v, layout, blk, scale, kb=None, ab=None, rpe=None):
    B, H, L, D = q.shape
    s = (q.float() @ k.float().transpose(-1, -2)) * scale + bs.token_bias(layout, blk, L, H, torch.float32, q.device)
    if rpe is not None:
        s = s + rpe.float().reshape(1, -1, L, L)
    if kb is not None:
        s = s + kb.float().view(B, 1, 1, L)
    if ab is not None:
        s = s + ab.float().view(1, 1, L, L)
    # a row with no allowed key has no softmax: its output (and every gradient through it) is zero, as in the kernel
    dead = torch.isneginf(s).all(-1, keepdim=True)
    return (torch.softmax(s.masked_fill(dead, 0.0), -1) @ v.float()).masked_fill(dead, 0.0)


def _grads_close(pairs, tag):
    for a, b, n in pairs:
        err = (a.float() - b).abs().max().item()
        assert err < 5e-2 * max(1.0, b.abs().max().item()), f"{tag} {n} err {err}"


@pytest.mark.parametrize("L", [4096, 16384])
def test_bert_padding_mask_in_kernel(L):
    """BERT-style additive key padding mask (0 keep / -10000 drop) applied inside the sparse kernels, forward and
    backward, against fp32 (reference `softmax.py:37-157`: key_padding_mask added per key inside the softmax)."""
    torch.manual_seed(3)
    B, H, D = 2, 4, 64
    cfg = FixedSparsityConfig(num_heads=H, block=64, num_local_blocks=4)
    layout = cfg.make_layout(L)
    q, k, v = (torch.randn(B, H, L, D, device="cuda").bfloat16().requires_grad_(True) for _ in range(3))
    lens = torch.tensor([L - 777, L // 2 + 5], device="cuda")
    kpm = torch.where(torch.arange(L, device="cuda")[None] < lens[:, None], 0.0, -10000.0)
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    o = bs.block_sparse_attention(q, k, v, layout, 64, key_padding_mask=kpm)
    do = torch.randn_like(o)
    o.backward(do)
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated() - base < 1024**3  # no [B, H, L, L] bias
    rows = slice(L // 2 - 64, L // 2 + 64)  # rows around sample 1's padding boundary, all keys
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    tok = layout.bool().repeat_interleave(64, 1).repeat_interleave(64, 2)[:, rows].cuda()
    s = (qr[:, :, rows] @ kr.transpose(-1, -2)) * D**-0.5
    s = s.masked_fill(~tok[None], float("-inf")) + kpm.view(B, 1, 1, L)
    ref = torch.softmax(s, -1) @ vr
    torch.testing.assert_close(o[:, :, rows].float(), ref, rtol=2e-2, atol=2e-2)
    ref.backward(do[:, :, rows].float())
    torch.testing.assert_close(q.grad[:, :, rows].float(), qr.grad[:, :, rows], rtol=5e-2, atol=5e-2)
    # padded keys receive no probability: their value gradient is exactly zero
    assert float(v.grad[1, :, L // 2 + 5:].abs().max()) == 0.0
    assert torch.isfinite(q.grad.float()).all() and torch.isfinite(k.grad.float()).all()


@pytest.mark.parametrize("what", ["kpm_mul", "attn_mask", "rpe", "rpe_shared", "all"])
def test_masks_and_rpe_in_kernel(what):
    torch.manual_seed(4)
    B, H, L, D = 2, 4, 1024, 64
    cfg = BigBirdSparsityConfig(num_heads=H, block=32)
    layout = cfg.make_layout(L)
    q, k, v = (torch.randn(B, H, L, D, device="cuda").bfloat16().requires_grad_(True) for _ in range(3))
    kw, rkw = {}, {}
    if what in ("kpm_mul", "all"):
        keep = (torch.rand(B, L, device="cuda") > 0.2).float()
        kw.update(key_padding_mask=keep, key_padding_mask_mode="mul")
        rkw["kb"] = torch.where(keep > 0, 0.0, float("-inf"))
    if what in ("attn_mask", "all"):
        am = torch.tril(torch.ones(L, L, device="cuda"))
        kw.update(attn_mask=am, attn_mask_mode="mul")
        rkw["ab"] = torch.where(am > 0, 0.0, float("-inf"))
    if what in ("rpe", "all"):
        kw["rpe"] = rkw["rpe"] = torch.randn(H, L, L, device="cuda")
    if what == "rpe_shared":
        kw["rpe"] = rkw["rpe"] = torch.randn(1, L, L, device="cuda")
    o = bs.block_sparse_attention(q, k, v, layout, 32, **kw)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _masked_ref(qr, kr, vr, layout, 32, D**-0.5, **rkw)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(ref)
    o.backward(do.bfloat16())
    ref.backward(do)
    assert torch.isfinite(q.grad.float()).all() and torch.isfinite(k.grad.float()).all()
    _grads_close(((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")), what)


@pytest.mark.parametrize("L,blk,dtype", [(192, 64, torch.bfloat16), (1000 - 8, 16, torch.float16),
                                         (320, 32, torch.float16)])
def test_fp16_and_unaligned_length(L, blk, dtype):
    """Sequence lengths that are a multiple of the block size but not of 128, and fp16 inputs (computed in bf16)."""
    torch.manual_seed(5)
    B, H, D = 2, 4, 64
    cfg = FixedSparsityConfig(num_heads=H, block=blk, num_local_blocks=4)
    layout = cfg.make_layout(L)
    q, k, v = (torch.randn(B, H, L, D, device="cuda").to(dtype).requires_grad_(True) for _ in range(3))
    assert bs.native_ok(q, k, v, blk)
    kpm = torch.zeros(B, L, device="cuda")
    kpm[1, L - 40:] = -10000.0
    o = bs.block_sparse_attention(q, k, v, layout, blk, key_padding_mask=kpm)
    assert o.dtype == dtype and o.shape == q.shape
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _masked_ref(qr, kr, vr, layout, blk, D**-0.5, kb=kpm)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(ref)
    o.backward(do.to(dtype))
    ref.backward(do)
    _grads_close(((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")), f"L={L}")


def test_sparse_self_attention_module_masks_stay_in_kernel(monkeypatch):
    """The module hands masks to the kernels: the dense [H, L, L] layout mask is never expanded on the device."""
    from deepspeedsyclsupport_amd.ops.sparse_attention.sparse_self_attention import SparseSelfAttention
    torch.manual_seed(6)
    B, H, L, D = 2, 4, 2048, 64
    cfg = FixedSparsityConfig(num_heads=H, block=64, num_local_blocks=4)
    attn = SparseSelfAttention(cfg, key_padding_mask_mode="add", attn_mask_mode="mul")
    monkeypatch.setattr(attn, "_block_mask", lambda *a, **k: pytest.fail("dense mask built on the device"))
    q, k, v = (torch.randn(B, H, L, D, device="cuda").half() for _ in range(3))
    kpm = torch.zeros(B, L, device="cuda")
    kpm[0, 1500:] = -10000.0
    am = torch.tril(torch.ones(L, L, device="cuda"))
    o = attn(q, k, v, key_padding_mask=kpm, attn_mask=am)
    ref = _masked_ref(q, k, v, attn.get_layout(L), 64, D**-0.5, kb=kpm, ab=torch.where(am > 0, 0.0, float("-inf")))
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
