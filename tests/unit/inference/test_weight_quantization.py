"""Weight-only post-init quantisation (reference `tests/unit/inference/quantization/test_intX_quantization.py`): the
codec's round-trip error bounds, module replacement by name key, tied weights, linear / embedding outputs against the
unquantised modules; on the GPU the same through the native group quantiser."""
from collections import OrderedDict

import pytest
import torch
import torch.nn as nn

from deepspeedsyclsupport_amd.inference.quantization import (DeQuantizer, QuantizedEmbedding, QuantizedLinear, Quantizer,
                                                            _init_group_wise_weight_quantization)


def _cfg(bits, gs=64, dim=1):
    return {"num_bits": bits, "group_size": gs, "group_dim": dim, "symmetric": False}


def _roundtrip(dtype, bits, device, dim=1):
    torch.manual_seed(1234)
    data = torch.randn(2048, 64, dtype=dtype, device=device)
    c = _cfg(bits, 64, dim)
    q, s, m = Quantizer(c).quantize(data)
    back = DeQuantizer(c, dtype).dequantize(q, s, m)
    assert back.shape == data.shape and back.dtype == dtype
    assert q.nbytes == data.numel() * bits // 8
    diff = (data.float() - back.float()).abs()
    # the reference's empirical thresholds
    assert diff.mean() < 0.15 and diff.max() < 0.5, (float(diff.mean()), float(diff.max()))
    return diff


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("dim", [0, 1])
def test_codec_roundtrip_cpu(bits, dtype, dim):
    d = _roundtrip(dtype, bits, "cpu", dim)
    if bits == 8 and dtype == torch.float32:
        assert d.max() < 0.03


def _model():
    torch.manual_seed(0)
    return nn.Sequential(OrderedDict((f"layer_{i}", nn.Linear(128, 128)) for i in range(5)))


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("dim", [0, 1])
def test_quantized_linear_cpu(bits, dim):
    model = _model()
    x = torch.randn(32, 128)
    with torch.no_grad():
        ref = model(x)
        cfg = {"weight_quantization": {"post_init_quant": {"layer": _cfg(bits, 64, dim)}}}
        model = _init_group_wise_weight_quantization(model, cfg)
        assert all(type(getattr(model, f"layer_{i}")) is QuantizedLinear for i in range(5))
        out = model(x)
    assert (ref - out).abs().mean() < 0.15
    if bits == 8:
        assert (ref - out).abs().mean() < 0.01
    sd = model.state_dict()
    assert "layer_0.q_codes" in sd and sd["layer_0.q_codes"].numel() == 128 * 128 * bits // 8


class _Tied(nn.Module):

    def __init__(self):
        super().__init__()
        self.embed_tokens = nn.Embedding(96, 64, padding_idx=0)
        self.fc = nn.Linear(64, 64)
        self.other = nn.Linear(64, 64)
        self.lm_head = nn.Linear(64, 96, bias=False)
        self.lm_head.weight = self.embed_tokens.weight

    def forward(self, ids):
        return self.lm_head(self.other(self.fc(self.embed_tokens(ids))))


@pytest.mark.parametrize("bits", [4, 8])
def test_keys_select_modules_and_tied_weights_share_codes(bits):
    torch.manual_seed(0)
    m = _Tied()
    ids = torch.randint(0, 96, (3, 7))
    with torch.no_grad():
        ref = m(ids)
        c = _cfg(bits, 32)
        _init_group_wise_weight_quantization(
            m, {"weight_quantization": {"post_init_quant": {"fc": c, "embed_tokens": c, "lm_head": c}}})
        assert type(m.fc) is QuantizedLinear and type(m.other) is nn.Linear
        assert type(m.embed_tokens) is QuantizedEmbedding and type(m.lm_head) is QuantizedLinear
        assert m.embed_tokens.q_codes.data_ptr() == m.lm_head.q_codes.data_ptr()
        out = m(ids)
        # the embedding dequantises only the looked-up rows and equals a lookup in the fully dequantised table
        full = m.embed_tokens.dequantized_weight()
        assert torch.equal(m.embed_tokens(ids), full[ids])
    tol = 0.02 if bits == 8 else 0.3
    assert (ref - out).abs().mean() < tol * ref.abs().mean() + tol
    with pytest.raises(AssertionError, match="multiple"):
        _init_group_wise_weight_quantization(
            _Tied(), {"weight_quantization": {"post_init_quant": {"fc": c, "f": c}}})


def test_quantized_initialization_covers_every_layer():
    m = _Tied()
    _init_group_wise_weight_quantization(m, {"weight_quantization": {"quantized_initialization": _cfg(8, 32)}})
    assert all(type(x) in (QuantizedLinear, QuantizedEmbedding) for x in (m.embed_tokens, m.fc, m.other, m.lm_head))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_codec_and_layers_gpu(bits, dtype):
    _roundtrip(dtype, bits, "cuda", 1)
    _roundtrip(dtype, bits, "cuda", 0)
    # the device codec agrees with the host one
    torch.manual_seed(3)
    w = torch.randn(256, 128, dtype=dtype)
    c = _cfg(bits, 64)
    qh, sh, mh = Quantizer(c).quantize(w)
    qd, sd, md = Quantizer(c).quantize(w.cuda())
    host = DeQuantizer(c, dtype).dequantize(qh, sh, mh).float()
    dev = DeQuantizer(c, dtype).dequantize(qd, sd, md).float().cpu()
    step = (w.float().view(-1, 64).amax(1) - w.float().view(-1, 64).amin(1)).max() / (2**bits - 1)
    assert (host - dev).abs().max() <= step * 1.01 + 1e-2
    model = _model().to("cuda", dtype)
    x = torch.randn(32, 128, dtype=dtype, device="cuda")
    with torch.no_grad():
        ref = model(x).float()
        _init_group_wise_weight_quantization(model, {"weight_quantization": {"post_init_quant": {"layer": c}}})
        out = model(x).float()
    assert (ref - out).abs().mean() < 0.15
    m = _Tied().to("cuda", dtype)
    ids = torch.randint(0, 96, (3, 7), device="cuda")
    with torch.no_grad():
        _init_group_wise_weight_quantization(m, {"weight_quantization": {"quantized_initialization": _cfg(bits, 32)}})
        assert torch.equal(m.embed_tokens(ids), m.embed_tokens.dequantized_weight()[ids])
        assert torch.isfinite(m(ids).float()).all()


def _init_quantized(out):
    import deepspeedsyclsupport_amd as ds
    torch.manual_seed(0)
    m = _Tied()
    ids = torch.randint(0, 96, (3, 7))
    with torch.no_grad():
        ref = m(ids)
    eng, *_ = ds.initialize(model=m, config={"train_micro_batch_size_per_gpu": 1,
                                             "weight_quantization": {"quantized_initialization": _cfg(8, 32)}})
    with torch.no_grad():
        got = eng.module(ids.to(eng.device)).cpu()
    torch.save({"kinds": [type(x).__name__ for x in (m.embed_tokens, m.fc, m.other, m.lm_head)],
                "err": float((got - ref).abs().mean() / ref.abs().mean())}, out)


def test_quantized_initialization_through_initialize(tmp_path):
    from ..common import run_distributed
    out = str(tmp_path / "r.pt")
    run_distributed(_init_quantized, 1, out)
    r = torch.load(out)
    assert r["kinds"] == ["QuantizedEmbedding", "QuantizedLinear", "QuantizedLinear", "QuantizedLinear"]
    assert r["err"] < 0.05
