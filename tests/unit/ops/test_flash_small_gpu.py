"""Small-head flash attention with biases / dropout (`csrc/attn/flash_small.hip`) against a plain fp32 PyTorch
reference of the same op — forward, dQ/dK/dV and both bias gradients (reference test:
`tests/unit/ops/deepspeed4science/test_DS4Sci_EvoformerAttention.py`, which compares against an fp32 einsum
attention with the same two biases)."""
import math

import pytest
import torch

from deepspeedsyclsupport_amd.ops import flash_small as FS

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def _case(Z, S, H, D, dtype, b1, b2, b2_div, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    q, k, v = (torch.randn(Z, S, H, D, device="cuda", dtype=dtype, generator=g) for _ in range(3))
    bias1 = (torch.randn(Z, S, device="cuda", generator=g) * 2).to(dtype) if b1 else None
    bias2 = torch.randn(Z // b2_div, H, S, S, device="cuda", generator=g).to(dtype) if b2 else None
    return q, k, v, bias1, bias2


@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("S,b1,b2,b2_div", [(128, True, True, 2), (100, True, True, 1), (200, False, True, 4),
                                            (64, True, False, 1), (130, False, False, 1)])
def test_fwd_bwd_vs_fp32(D, dtype, S, b1, b2, b2_div):
    Z, H = 4, 3
    q, k, v, bias1, bias2 = _case(Z, S, H, D, dtype, b1, b2, b2_div)
    ins = [t.detach().clone().requires_grad_(True) if t is not None else None for t in (q, k, v, bias1, bias2)]
    out = FS.flash_small(*ins[:3], ins[3], ins[4], b2_div=b2_div)
    refs = [t.detach().float().clone().requires_grad_(True) if t is not None else None for t in (q, k, v, bias1, bias2)]
    ref = FS.reference(*refs[:3], refs[3], refs[4], b2_div=b2_div)
    tol = 2e-2 if dtype == torch.bfloat16 else 6e-3
    assert _rel(out, ref) < tol
    go = torch.randn_like(ref)
    out.backward(go.to(dtype))
    ref.backward(go)
    for name, a, r in zip(("dq", "dk", "dv", "db1", "db2"), ins, refs):
        if a is None:
            continue
        assert a.grad is not None, name
        assert _rel(a.grad, r.grad) < 2 * tol, (name, _rel(a.grad, r.grad))


@pytest.mark.parametrize("D", [32, 64])
def test_dropout_matches_host_mask(D):
    Z, S, H, p, seed = 2, 160, 2, 0.25, 12345
    q, k, v, bias1, _ = _case(Z, S, H, D, torch.bfloat16, True, False, 1, seed=3)
    ins = [t.detach().clone().requires_grad_(True) for t in (q, k, v)]
    out = FS.flash_small(*ins, bias1, dropout_p=p, seed=seed)
    keep = FS.keep_mask(seed, Z, H, S, p)
    frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01
    refs = [t.detach().float().clone().requires_grad_(True) for t in (q, k, v)]
    ref = FS.reference(*refs, bias1, keep=keep, p=p)
    assert _rel(out, ref) < 2e-2
    go = torch.randn_like(ref)
    out.backward(go.bfloat16())
    ref.backward(go)
    for a, r in zip(ins, refs):
        assert _rel(a.grad, r.grad) < 4e-2
    # same seed -> same output; new seed -> different
    again = FS.flash_small(q, k, v, bias1, dropout_p=p, seed=seed)
    assert torch.equal(again, out.detach())
    other = FS.flash_small(q, k, v, bias1, dropout_p=p, seed=seed + 1)
    assert not torch.equal(other, out.detach())


@pytest.mark.parametrize("D", [32, 64])
def test_evoformer_api_kernel_vs_sdpa(D):
    from deepspeedsyclsupport_amd.ops import deepspeed4science as E
    B, N, S, H = 1, 3, 96, 4
    g = torch.Generator(device="cuda").manual_seed(1)
    Q, K, V = (torch.randn(B, N, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    mask = (torch.rand(B, N, 1, 1, S, device="cuda", generator=g) > 0.2).to(torch.bfloat16)
    b1 = (1e9 * (mask - 1)).to(torch.bfloat16)
    b2 = torch.randn(B, 1, H, S, S, device="cuda", dtype=torch.bfloat16, generator=g)
    ins = [t.clone().requires_grad_(True) for t in (Q, K, V, b1, b2)]
    out = E.DS4Sci_EvoformerAttention(ins[0], ins[1], ins[2], [ins[3], ins[4]])
    refs = [t.float().clone().requires_grad_(True) for t in (Q, K, V, b1, b2)]
    ref = E._sdpa_path(refs[0], refs[1], refs[2], [refs[3], refs[4]])
    assert out.shape == (B, N, S, H, D)
    assert _rel(out, ref) < 2e-2
    go = torch.randn_like(ref)
    out.backward(go.bfloat16())
    ref.backward(go)
    for name, a, r in zip(("dq", "dk", "dv", "db2"), ins[:3] + ins[4:], refs[:3] + refs[4:]):
        assert _rel(a.grad, r.grad) < 4e-2, name
    assert ins[3].grad is not None


def test_bert_layer_uses_kernel_with_mask():
    from deepspeedsyclsupport_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
    torch.manual_seed(0)
    cfg = DeepSpeedTransformerConfig(batch_size=2, hidden_size=256, heads=4, attn_dropout_ratio=0.0,
                                     hidden_dropout_ratio=0.0, num_hidden_layers=2, initializer_range=0.02)
    layer = DeepSpeedTransformerLayer(cfg).cuda().to(torch.bfloat16)
    x = torch.randn(2, 96, 256, device="cuda", dtype=torch.bfloat16)
    m = torch.zeros(2, 1, 1, 96, device="cuda")
    m[1, ..., 80:] = -10000.0
    calls = []
    orig = FS.FlashSmallFunc.apply

    def spy(*a):
        calls.append(1)
        return orig(*a)

    FS.FlashSmallFunc.apply = spy
    try:
        out = layer(x, m)
    finally:
        FS.FlashSmallFunc.apply = orig
    assert calls, "the BERT layer did not take the fused attention kernel"
    ref_layer = DeepSpeedTransformerLayer(cfg).cuda().float()
    ref_layer.load_state_dict({k: v.float() for k, v in layer.state_dict().items()})
    ref = ref_layer(x.float(), m)
    assert _rel(out, ref) < 3e-2


@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("Sk", [77, 64, 300])
def test_cross_length_forward(D, Sk):
    """Queries and keys of different lengths (diffusers cross-attention): forward only, with a per-key bias."""
    Z, S, H = 2, 150, 2
    g = torch.Generator(device="cuda").manual_seed(5)
    q = torch.randn(Z, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
    k, v = (torch.randn(Z, Sk, H, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(2))
    b1 = torch.randn(Z, Sk, device="cuda", generator=g).bfloat16()
    with torch.no_grad():
        out = FS.flash_small(q, k, v, b1)
    assert _rel(out, FS.reference(q, k, v, b1)) < 2e-2
    with pytest.raises(NotImplementedError):
        FS.flash_small(q.requires_grad_(True), k, v)
