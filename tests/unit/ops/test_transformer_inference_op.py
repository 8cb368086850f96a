"""Op-level inference layer (`ops/transformer/inference`, reference `tests/unit/ops/transformer/inference/`):
the standalone DeepSpeedTransformerInference layer against a plain PyTorch fp32 pre-LN decoder block, and
prefill + cached decode through `layer_past` against the full-sequence forward."""
import math

import pytest
import torch
import torch.nn.functional as F

from deepspeedsyclsupport_amd.ops.transformer.inference import (DeepSpeedInferenceConfig,
                                                                DeepSpeedMoEInference, DeepSpeedMoEInferenceConfig,
                                                                DeepSpeedTransformerInference)
from deepspeedsyclsupport_amd.utils.types import ActivationFuncType, NormType


def _ref_block(layer, x, heads):
    L = layer.layer
    B, n, H = x.shape
    D = H // heads
    a = F.layer_norm(x, (H, ), L.ln1_w.float(), L.ln1_b.float(), 1e-5)
    q, k, v = F.linear(a, L.qkv_w.float(), L.qkv_b.float()).split(H, dim=-1)
    q, k, v = (t.view(B, n, heads, D).transpose(1, 2) for t in (q, k, v))
    att = (q @ k.transpose(-1, -2)) / math.sqrt(D)
    att = att.masked_fill(torch.ones(n, n, dtype=torch.bool).triu(1), float("-inf")).softmax(-1)
    o = (att @ v).transpose(1, 2).reshape(B, n, H)
    x = x + F.linear(o, L.o_w.float(), L.o_b.float())
    m = F.layer_norm(x, (H, ), L.ln2_w.float(), L.ln2_b.float(), 1e-5)
    m = F.linear(F.gelu(F.linear(m, L.fc1_w.float(), L.fc1_b.float())), L.fc2_w.float(), L.fc2_b.float())
    return x + m


def _cfg(**kw):
    base = dict(hidden_size=64, intermediate_size=256, heads=4, num_hidden_layers=1, layer_norm_eps=1e-5,
                dtype=torch.float32, max_out_tokens=128, mlp_act_func_type=ActivationFuncType.GELU)
    base.update(kw)
    return DeepSpeedInferenceConfig(**base)


def test_layer_matches_reference_block():
    torch.manual_seed(0)
    layer = DeepSpeedTransformerInference(_cfg(), device="cpu")
    with torch.no_grad():
        for p in layer.layer.parameters():
            if p.dim() == 1:
                p.normal_(0.0, 0.1).add_(1.0 if p.shape[0] == 64 else 0.0)
    x = torch.randn(2, 9, 64)
    out = layer(x)[0]
    torch.testing.assert_close(out, _ref_block(layer, x, 4), atol=2e-5, rtol=2e-5)


@pytest.mark.parametrize("rotary", [-1, 16])
def test_layer_past_decode_matches_full_forward(rotary):
    torch.manual_seed(1)
    layer = DeepSpeedTransformerInference(_cfg(rotary_dim=rotary, rotate_half=True), device="cpu")
    x = torch.randn(2, 12, 64)
    full, _ = layer(x, use_cache=True)
    out, past = layer(x[:, :8], use_cache=True)
    assert past[0].shape == (2, 4, 8, 16)
    torch.testing.assert_close(out, full[:, :8], atol=1e-5, rtol=1e-5)
    for t in range(8, 12):
        out, past = layer(x[:, t:t + 1], layer_past=past, use_cache=True)
        torch.testing.assert_close(out[:, 0], full[:, t], atol=1e-5, rtol=1e-5)
    assert past[0].shape[2] == 12


def test_config_lowering_and_guards():
    spec = _cfg(norm_type=NormType.RMSNorm, mlp_act_func_type=ActivationFuncType.GATED_SILU, rotary_dim=16,
                num_kv=2, bigscience_bloom=False).to_spec()
    assert (spec.norm, spec.act, spec.gated_mlp, spec.pos, spec.num_kv_heads) == ("rms", "silu", True, "rope_gptj", 2)
    assert _cfg(bigscience_bloom=True).to_spec().pos == "alibi"
    with pytest.raises(ValueError):
        _cfg(use_triton=True)
    with pytest.raises(ValueError):
        DeepSpeedTransformerInference(_cfg(max_out_tokens=16), device="cpu")(torch.randn(1, 80, 64))


def test_moe_layer_runs():
    torch.manual_seed(2)
    cfg = DeepSpeedMoEInferenceConfig(hidden_size=64, intermediate_size=128, heads=4, num_hidden_layers=1,
                                      moe_experts=4, k=2, max_out_tokens=64)
    layer = DeepSpeedMoEInference(cfg, device="cpu")
    assert layer.layer.fc1_w.shape[0] == 4
    out = layer(torch.randn(1, 5, 64))[0]
    assert out.shape == (1, 5, 64) and torch.isfinite(out).all()


@pytest.mark.gpu
def test_layer_bf16_gpu_prefill_and_decode():
    """bf16 on MI355X: fused QKV/RoPE/paged-append epilogue, flash prefill and paged decode vs fp32 CPU layer."""
    torch.manual_seed(3)
    cfg = dict(hidden_size=1024, intermediate_size=4096, heads=8, rotary_dim=128, rotate_half=True,
               norm_type=NormType.RMSNorm, mlp_act_func_type=ActivationFuncType.GATED_SILU, max_out_tokens=256)
    ref = DeepSpeedTransformerInference(_cfg(**cfg), device="cpu")
    gpu = DeepSpeedTransformerInference(_cfg(**dict(cfg, dtype=torch.bfloat16)), device="cuda")
    with torch.no_grad():
        for p in ref.layer.parameters():  # round the reference to bf16 so both see identical weights
            p.copy_(p.bfloat16().float())
        for a, b in zip(ref.layer.parameters(), gpu.layer.parameters()):
            b.copy_(a)
    x = torch.randn(2, 40, 1024).bfloat16().float()
    full = ref(x)[0]
    out, past = gpu(x[:, :36].cuda().bfloat16(), use_cache=True)
    torch.testing.assert_close(out.float().cpu(), full[:, :36], atol=5e-2, rtol=5e-2)
    for t in range(36, 40):
        out, past = gpu(x[:, t:t + 1].cuda().bfloat16(), layer_past=past, use_cache=True)
        torch.testing.assert_close(out[:, 0].float().cpu(), full[:, t], atol=5e-2, rtol=5e-2)


def test_bloom_alibi_and_gqa_decode_consistency():
    """ALiBi (bigscience_bloom) and grouped KV heads: cached decode reproduces the full-sequence forward."""
    torch.manual_seed(4)
    for kw in (dict(bigscience_bloom=True), dict(num_kv=2, rotary_dim=16, rotate_half=True)):
        layer = DeepSpeedTransformerInference(_cfg(**kw), device="cpu")
        x = torch.randn(1, 10, 64)
        full = layer(x)[0]
        out, past = layer(x[:, :7], use_cache=True)
        assert past[0].shape[1] == (2 if "num_kv" in kw else 4)
        for t in range(7, 10):
            out, past = layer(x[:, t:t + 1], layer_past=past, use_cache=True)
            torch.testing.assert_close(out[:, 0], full[:, t], atol=1e-5, rtol=1e-5)
