"""gfx950 flash-attention forward (csrc/attn/flash_fwd.hip) against an fp32 PyTorch reference, plus the autograd
path (our O/LSE through the efficient-attention backward) against fp32 SDPA gradients."""
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
