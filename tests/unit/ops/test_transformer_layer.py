"""DeepSpeedTransformerLayer vs a plain-PyTorch BERT layer with identical weights (reference
`tests/unit/ops/accelerators/test_accelerator_forward.py` / `_backward.py` compare against HF BertLayer)."""
import math

import pytest
import torch
import torch.nn.functional as F

from deepspeedsyclsupport_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer


def _ref(layer, x, mask, pre_ln):
    c = layer.config
    B, S, H = x.shape
    nh = c.heads

    def ln(t, w, b):
        return F.layer_norm(t, (H, ), w, b, c.layer_norm_eps)

    def attn(t):
        qkv = F.linear(t, layer.attn_qkvw, layer.attn_qkvb).view(B, S, 3, nh, H // nh).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        s = q @ k.transpose(-1, -2) / math.sqrt(H // nh) + mask
        ctx = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, H)
        return F.linear(ctx, layer.attn_ow, layer.attn_ob)

    def ff(t):
        return F.linear(F.gelu(F.linear(t, layer.inter_w, layer.inter_b)), layer.output_w, layer.output_b)

    if pre_ln:
        r = x + attn(ln(x, layer.attn_nw, layer.attn_nb))
        return r + ff(ln(r, layer.norm_w, layer.norm_b))
    r = ln(x + attn(x), layer.attn_nw, layer.attn_nb)
    return ln(r + ff(r), layer.norm_w, layer.norm_b)


def _run(pre_ln, device, dtype, tol):
    torch.manual_seed(0)
    cfg = DeepSpeedTransformerConfig(batch_size=2, hidden_size=64, heads=4, attn_dropout_ratio=0.0,
                                     hidden_dropout_ratio=0.0, num_hidden_layers=2, initializer_range=0.05,
                                     pre_layer_norm=pre_ln, layer_norm_eps=1e-12)
    layer = DeepSpeedTransformerLayer(cfg).to(device=device, dtype=dtype)
    with torch.no_grad():
        for p in (layer.attn_nb, layer.norm_b, layer.attn_qkvb, layer.inter_b):
            p.normal_(0, 0.1)
    x = torch.randn(2, 16, 64, device=device, dtype=dtype, requires_grad=True)
    mask = torch.zeros(2, 1, 1, 16, device=device, dtype=dtype)
    mask[1, ..., 12:] = -10000.0
    out = layer(x, mask)
    ref = _ref(layer, x, mask, pre_ln)
    torch.testing.assert_close(out.float(), ref.float(), rtol=tol, atol=tol)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, [x, layer.attn_qkvw, layer.norm_w], g)
    gb = torch.autograd.grad(ref, [x, layer.attn_qkvw, layer.norm_w], g)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a.float(), b.float(), rtol=tol * 5, atol=tol * 5)


@pytest.mark.parametrize("pre_ln", [True, False])
def test_transformer_layer_cpu(pre_ln):
    _run(pre_ln, "cpu", torch.float32, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("pre_ln", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_transformer_layer_gpu(pre_ln, dtype):
    _run(pre_ln, "cuda", dtype, 2e-3 if dtype == torch.float32 else 5e-2)
