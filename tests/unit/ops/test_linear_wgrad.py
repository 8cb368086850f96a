"""Training linear (`ops/linear.py`): the K-major weight-gradient path (HIP transpose + TN GEMM) against
nn.Linear autograd, and the transpose kernel against torch."""
import pytest
import torch

from deepspeedsyclsupport_amd.ops import linear as L


def test_linear_function_matches_autograd_cpu():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 16, requires_grad=True)
    lin = torch.nn.Linear(16, 8)
    y = L.linear(x, lin.weight, lin.bias)
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, lin.weight, lin.bias), g)
    x2 = x.detach().clone().requires_grad_(True)
    y2 = lin(x2)
    rx, rw, rb = torch.autograd.grad(y2, (x2, lin.weight, lin.bias), g)
    torch.testing.assert_close(y, y2)
    torch.testing.assert_close(gx, rx)
    torch.testing.assert_close(gw, rw)
    torch.testing.assert_close(gb, rb)


@pytest.mark.gpu
@pytest.mark.parametrize("R,C,ld", [(64, 64, 64), (8192, 4104, 4104), (136, 4096, 4200), (32760, 512, 512)])
def test_transpose16(R, C, ld):
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    base = torch.randn(R, ld, device="cuda").bfloat16()
    x = base[:, :C]
    torch.testing.assert_close(hip_ops().transpose16(x), x.t().contiguous(), rtol=0, atol=0)
    p = hip_ops().transpose16(x, R + 40)
    torch.testing.assert_close(p[:, :R], x.t(), rtol=0, atol=0)
    assert (p[:, R:] == 0).all()


@pytest.mark.gpu
def test_kmajor_weight_grad_gpu():
    torch.manual_seed(0)
    T, n_in, n_out = 8200, 512, 384
    x = torch.randn(T, n_in, device="cuda").bfloat16().requires_grad_(True)
    w = (torch.randn(n_out, n_in, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    assert L._kmajor_ok(torch.empty(T, n_out, device="cuda", dtype=torch.bfloat16), x)
    y = L.linear(x, w)
    g = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, (x, w), g)
    ref = g.float().t() @ x.float()
    assert ((gw.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    torch.testing.assert_close(gx.float(), (g.float() @ w.float()), rtol=2e-2, atol=2e-1)


def test_linear_function_under_autocast_cpu():
    lin = torch.nn.Linear(16, 8)
    x = torch.randn(4, 16, requires_grad=True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        y = L.linear(x, lin.weight, lin.bias)
    y.float().sum().backward()
    assert lin.weight.grad.dtype == torch.float32 and x.grad.dtype == torch.float32


@pytest.mark.gpu
@pytest.mark.parametrize("T,I", [(8192, 704), (8200, 1024)])
def test_gated_activation_kmajor_side_outputs(T, I):
    """The gated activation of a long token batch writes the token-contiguous copies itself: the values equal the
    plain kernels', the down projection keeps only the K-major copy, and neither weight gradient of the
    gate_up -> act -> down chain goes through the separate transpose pass."""
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(0)
    gu = torch.randn(T, 2 * I, device="cuda").bfloat16()
    out, out_t = hip_ops().gated_act_fwd_t(gu, 0, 256)
    ref = hip_ops().gated_act_fwd(gu, 0)
    Tp = -(-T // 256) * 256
    assert out_t.shape == (I, Tp)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    torch.testing.assert_close(out_t[:, :T], ref.t(), rtol=0, atol=0)
    assert (out_t[:, T:] == 0).all()
    d = torch.randn(T, I, device="cuda").bfloat16()
    dgu, dgu_t = hip_ops().gated_act_bwd_t(d, gu, 0, 256)
    dref = hip_ops().gated_act_bwd(d, gu, 0)
    torch.testing.assert_close(dgu, dref, rtol=0, atol=0)
    torch.testing.assert_close(dgu_t[:, :T], dref.t(), rtol=0, atol=0)
    assert (dgu_t[:, T:] == 0).all()
    # end to end through autograd: x -> gate_up linear -> gated act -> down linear
    H = 256
    x = torch.randn(T, H, device="cuda").bfloat16().requires_grad_(True)
    w1 = (torch.randn(2 * I, H, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    w2 = (torch.randn(H, I, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    before = dict(L.STATS)
    y = L.linear(DF.gated_activation(L.linear(x, w1), "silu"), w2)
    g = torch.randn_like(y)
    gx, g1, g2 = torch.autograd.grad(y, (x, w1, w2), g)
    # w2's x operand and w1's gradient operand came from the producer kernels (2), x of w1 and dY of w2 did not (2)
    assert L.STATS["kmajor_from_producer"] - before["kmajor_from_producer"] == 2
    assert L.STATS["kmajor_transposed"] - before["kmajor_transposed"] == 2
    xf, w1f, w2f = x.detach().float().requires_grad_(True), w1.detach().float().requires_grad_(True), \
        w2.detach().float().requires_grad_(True)
    h = xf @ w1f.t()
    a = torch.nn.functional.silu(h[:, :I]) * h[:, I:]
    yr = a @ w2f.t()
    rx, r1, r2 = torch.autograd.grad(yr, (xf, w1f, w2f), g.float())
    for got, want in ((g1, r1), (g2, r2), (gx, rx)):
        assert ((got.float() - want).abs().max() / want.abs().max()).item() < 3e-2
