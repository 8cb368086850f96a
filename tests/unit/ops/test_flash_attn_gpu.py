"""gfx950 flash attention (csrc/attn/flash_fwd.hip, flash_bwd.hip) against fp32 PyTorch references: forward O/LSE,
and the in-tree backward's dq/dk/dv against fp32 autograd (GQA 1:1 .. 8:1, causal and full, ragged lengths,
strided views, long sequences)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def ref_attn(q, k, v, causal, scale):
    rep = q.shape[1] // k.shape[1]
    k = k.float().repeat_interleave(rep, 1)
    v = v.float().repeat_interleave(rep, 1)
    s = (q.float() @ k.transpose(-1, -2)) * scale
    if causal:
        S, T = s.shape[-2:]
        s = s.masked_fill(torch.ones(S, T, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    return torch.softmax(s, -1) @ v, lse


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,Hq,Hk,S", [(1, 2, 2, 128), (2, 4, 4, 1000), (1, 8, 2, 512), (2, 2, 2, 2048),
                                       (1, 1, 1, 64), (1, 2, 1, 200)])
def test_flash_fwd(causal, B, Hq, Hk, S):
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(0)
    q = torch.randn(B, Hq, S, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(128)
    o, lse = hip_ops().flash_fwd(q, k, v, causal, scale, True)
    ro, rlse = ref_attn(q, k, v, causal, scale)
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, rlse, rtol=1e-3, atol=1e-3)
    assert o.transpose(1, 2).is_contiguous()  # memory is [B,S,H,D]


def test_flash_fwd_strided_inputs():
    """q/k/v as views of a packed [B,S,H,D] buffer (non-contiguous head-major views)."""
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(1)
    B, S, H = 2, 384, 4
    qkv = torch.randn(B, S, 3 * H, 128, device="cuda", dtype=torch.bfloat16)
    q, k, v = (t.transpose(1, 2) for t in qkv.split(H, dim=2))
    o, lse = hip_ops().flash_fwd(q, k, v, True, 0.1, True)
    ro, rlse = ref_attn(q, k, v, True, 0.1)
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("Hq,Hk", [(4, 4), (4, 2)])
def test_flash_autograd(Hq, Hk):
    from deepspeedsyclsupport_amd.ops.attention import attention, flash_supported
    torch.manual_seed(2)
    B, S = 2, 512
    q = torch.randn(B, Hq, S, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    assert flash_supported(q, k, v)
    o = attention(q, k, v, causal=True)
    g = torch.randn_like(o)
    o.backward(g)
    q32, k32, v32 = (t.detach().float().requires_grad_() for t in (q, k, v))
    ro, _ = ref_attn(q32, k32, v32, True, 128**-0.5)
    ro.backward(g.float())
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)
    for a, b in ((q.grad, q32.grad), (k.grad, k32.grad), (v.grad, v32.grad)):
        torch.testing.assert_close(a.float(), b, rtol=5e-2, atol=5e-2)


def _bwd_case(B, Hq, Hk, S, causal, seed=3, strided=False):
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(seed)
    if strided:  # q/k/v as [B,H,S,D] views of one packed [B,S,Hq+2Hk,D] buffer, dout token-major too
        qkv = torch.randn(B, S, Hq + 2 * Hk, 128, device="cuda", dtype=torch.bfloat16)
        q, k, v = (t.transpose(1, 2) for t in qkv.split([Hq, Hk, Hk], dim=2))
        do = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    else:
        q = torch.randn(B, Hq, S, 128, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16)
        do = torch.randn(B, Hq, S, 128, device="cuda", dtype=torch.bfloat16)
    scale = 128**-0.5
    o, lse = hip_ops().flash_fwd(q, k, v, causal, scale, True)
    dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, scale, 1 if causal else 0)
    q32, k32, v32 = (t.detach().float().requires_grad_() for t in (q, k, v))
    ro, _ = ref_attn(q32, k32, v32, causal, scale)
    ro.backward(do.float())
    for name, a, b in (("dq", dq, q32.grad), ("dk", dk, k32.grad), ("dv", dv, v32.grad)):
        err = (a.float() - b).abs().max().item()
        ref = b.abs().max().item()
        assert err <= 2e-2 * ref + 2e-2, (name, err, ref)
        torch.testing.assert_close(a.float(), b, rtol=5e-2, atol=5e-2 * max(1.0, ref / 8))
    assert dq.shape == q.shape and dk.shape == k.shape and dv.shape == v.shape


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,Hq,Hk,S", [(1, 2, 2, 256), (2, 4, 4, 512), (1, 8, 1, 512), (1, 8, 2, 384),
                                       (2, 2, 2, 100), (1, 4, 1, 1000), (1, 1, 1, 32)])
def test_flash_bwd(causal, B, Hq, Hk, S):
    _bwd_case(B, Hq, Hk, S, causal)


def test_flash_bwd_strided():
    _bwd_case(2, 4, 2, 640, True, strided=True)


@pytest.mark.parametrize("Hq,Hk", [(2, 2), (8, 1)])
def test_flash_bwd_long(Hq, Hk):
    # fp32 reference at 8k: [Hq, S, S] fp32 scores = 2 GB at Hq 8; keep B=1
    _bwd_case(1, Hq, Hk, 8192, True, seed=5)


def test_flash_bwd_32k():
    """The Ulysses per-GPU shape class: one head at 32k tokens, compared in row chunks to bound reference memory."""
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(6)
    S = 32768
    q, k, v, do = (torch.randn(1, 1, S, 128, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    scale = 128**-0.5
    o, lse = hip_ops().flash_fwd(q, k, v, True, scale, True)
    dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, scale, 1)
    # reference dq for the last 256 query rows (they see every key), and dk/dv for the last 256 keys (seen by only
    # the queries at and after them)
    kf, vf = k[0, 0].float(), v[0, 0].float()
    qs, dos = q[0, 0, -256:].float(), do[0, 0, -256:].float()
    s = (qs @ kf.T) * scale
    qi = torch.arange(S - 256, S, device="cuda")[:, None]
    s = s.masked_fill(torch.arange(S, device="cuda")[None, :] > qi, float("-inf"))
    p = torch.softmax(s, -1)
    dp = dos @ vf.T
    delta = (p * dp).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    ref_dq = (ds @ kf) * scale
    torch.testing.assert_close(dq[0, 0, -256:].float(), ref_dq, rtol=5e-2, atol=5e-2)
    # last 256 keys: only the last 256 queries attend to them
    dv_ref = p[:, -256:].T @ dos
    dk_ref = (ds[:, -256:].T @ qs) * scale
    torch.testing.assert_close(dv[0, 0, -256:].float(), dv_ref, rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(dk[0, 0, -256:].float(), dk_ref, rtol=5e-2, atol=5e-2)


def test_flash_bwd_deterministic_shapes_no_nan():
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(7)
    q = torch.randn(1, 4, 300, 128, device="cuda", dtype=torch.bfloat16) * 8
    k = torch.randn(1, 4, 300, 128, device="cuda", dtype=torch.bfloat16) * 8
    v = torch.randn(1, 4, 300, 128, device="cuda", dtype=torch.bfloat16)
    do = torch.randn_like(q)
    o, lse = hip_ops().flash_fwd(q, k, v, True, 0.088, True)
    dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, 0.088, 1)
    assert all(torch.isfinite(t).all() for t in (dq, dk, dv))
