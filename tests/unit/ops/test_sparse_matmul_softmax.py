"""Standalone block-sparse MatMul (sdd / dsd / dds) and Softmax (`ops/sparse_attention/{matmul,softmax}.py`;
reference `matmul.py:628`, `softmax.py:224`) against dense PyTorch with the layout applied as a mask, including the
three-step attention they compose to and its gradients."""
import pytest
import torch

from deepspeedsyclsupport_amd.ops.sparse_attention.matmul import MatMul
from deepspeedsyclsupport_amd.ops.sparse_attention.softmax import Softmax

B, H, L, D, BLK = 2, 3, 64, 16, 16


def _layout():
    g = torch.Generator().manual_seed(0)
    lay = (torch.rand(H, L // BLK, L // BLK, generator=g) < 0.5).long()
    for h in range(H):
        lay[h].fill_diagonal_(1)
    return lay


def _to_dense(sp, lay, fill=0.0):
    out = torch.full((sp.shape[0], H, L, L), fill, dtype=sp.dtype)
    for n, (h, i, j) in enumerate(lay.nonzero().tolist()):
        out[:, h, i * BLK:(i + 1) * BLK, j * BLK:(j + 1) * BLK] = sp[:, n]
    return out


def test_three_modes_and_transposes():
    lay = _layout()
    torch.manual_seed(1)
    q, k = torch.randn(B, H, L, D), torch.randn(B, H, L, D)
    mask = lay.repeat_interleave(BLK, 1).repeat_interleave(BLK, 2)[None].float()
    sdd = MatMul(lay, BLK, "sdd", trans_b=True)(q, k)
    assert sdd.shape == (B, int(lay.sum()), BLK, BLK)
    torch.testing.assert_close(_to_dense(sdd, lay), (q @ k.transpose(-1, -2)) * mask, rtol=1e-4, atol=1e-4)
    v = torch.randn(B, H, L, D)
    dsd = MatMul(lay, BLK, "dsd")(sdd, v)
    torch.testing.assert_close(dsd, ((q @ k.transpose(-1, -2)) * mask) @ v, rtol=1e-4, atol=1e-3)
    dsd_t = MatMul(lay, BLK, "dsd", trans_a=True)(sdd, v)
    torch.testing.assert_close(dsd_t, ((q @ k.transpose(-1, -2)) * mask).transpose(-1, -2) @ v, rtol=1e-4, atol=1e-3)
    x = torch.randn(B, H, D, L)
    dds = MatMul(lay, BLK, "dds")(x, sdd)
    torch.testing.assert_close(dds, x @ ((q @ k.transpose(-1, -2)) * mask), rtol=1e-4, atol=1e-3)
    with pytest.raises(NotImplementedError):
        MatMul(lay, BLK, "ddd")


def test_softmax_with_masks_and_attention_gradients():
    lay = _layout()
    torch.manual_seed(2)
    q, k, v = (torch.randn(B, H, L, D, requires_grad=True) for _ in range(3))
    rpe = torch.randn(H, L, L) * 0.1
    kp = torch.zeros(B, L)
    kp[1, -9:] = float("-inf")
    am = torch.ones(L, L).tril()
    scale = D**-0.5
    sm = Softmax(lay, BLK)
    scores = MatMul(lay, BLK, "sdd", trans_b=True)(q, k)
    probs = sm(scores, scale=scale, rpe=rpe, key_padding_mask=kp, attn_mask=am, attn_mask_mode="mul")
    out = MatMul(lay, BLK, "dsd")(probs, v)

    qr, kr, vr = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    dense = (qr @ kr.transpose(-1, -2)) * scale + rpe[None] + kp[:, None, None, :]
    blocked = lay.repeat_interleave(BLK, 1).repeat_interleave(BLK, 2)[None].bool() & am.bool()[None, None]
    dense = dense.masked_fill(~blocked, float("-inf"))
    ref = torch.softmax(dense, -1) @ vr
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(_to_dense(probs, lay).sum(-1), torch.ones(B, H, L), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(ref)
    (out * g).sum().backward()
    (ref * g).sum().backward()
    for a, b_ in ((q, qr), (k, kr), (v, vr)):
        torch.testing.assert_close(a.grad, b_.grad, rtol=1e-3, atol=1e-4)
    with pytest.raises(ValueError):
        sm(scores, attn_mask=am, attn_mask_mode="xor")
