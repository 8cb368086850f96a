"""bf16 decode GEMV over the pre-shuffled weight (`ops/bf16_gemv.py`, `csrc/gemv/skinny_bf16_sh.hip`): layout round
trip on the host; on the GPU the MFMA stream, its un-finalized form with the fused consumers, the un-shuffle kernel
and HIP-graph replays (the split-K workspace must come back to zero every time) against fp32 references."""
import pytest
import torch

from deepspeedsyclsupport_amd.ops.bf16_gemv import Bf16Weight, preshuffle16, unshuffle16


@pytest.mark.parametrize("N,K", [(16, 64), (37, 128), (4096, 256)])
def test_shuffle_round_trip_cpu(N, K):
    torch.manual_seed(0)
    w = torch.randn(N, K).bfloat16()
    sh = preshuffle16(w)
    assert sh.shape == ((N + 15) // 16, K // 64, 2, 64, 8)
    assert torch.equal(unshuffle16(sh, N), w)
    # element addressing as documented: wsh[nb, kq, h, lane, j] = w[16 nb + lane % 16, 64 kq + 16 (lane // 16) + 8 h + j]
    nb, kq, h, lane, j = 0, K // 64 - 1, 1, 37, 5
    assert sh[nb, kq, h, lane, j] == w[16 * nb + lane % 16, 64 * kq + 16 * (lane // 16) + 8 * h + j]
    bw = Bf16Weight(w)
    assert torch.equal(bw.materialize(), w)
    x = torch.randn(3, K).bfloat16()
    torch.testing.assert_close(bw.linear(x).float(), x.float() @ w.float().t(), rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 8, 13, 16])
@pytest.mark.parametrize("N,K", [(4096, 4096), (333, 11008), (100, 256), (12288, 4096), (4096, 11008), (50, 64)])
@pytest.mark.parametrize("cfg", [1, 2, 3, 4])
def test_bf16_sh_gemv_gpu(M, N, K, cfg):
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(M * 1000 + N)
    hip_ops().skinny_b16_tune(cfg, 0)
    try:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        bw = Bf16Weight(w)
        ref = x.float() @ w.float().t()
        for _ in range(2):  # the second call starts from the workspace the first one re-zeroed
            y = bw.linear(x, b)
            torch.testing.assert_close(y.float(), ref + b.float(), rtol=2e-2, atol=2e-2)
        y0 = bw.raw(x, None).finalize()
        torch.testing.assert_close(y0.float(), ref, rtol=2e-2, atol=2e-2)
        assert torch.equal(hip_ops().unshuffle_sh16(bw.wsh, N), w)
    finally:
        hip_ops().skinny_b16_tune(0, 0)


@pytest.mark.gpu
def test_bf16_sh_fused_consumers_and_graph():
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(5)
    M, K, N = 4, 4096, 4096
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
    wg = (torch.randn(2 * 1024, K, device="cuda") * 0.03).bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()
    nw = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16()
    bw, bg = Bf16Weight(w), Bf16Weight(wg)
    # projection + residual + RMSNorm in one finalize
    y, r = bw.raw(x).finalize_rms(res, nw, 1e-5)
    h = x.float() @ w.float().t() + res.float()
    torch.testing.assert_close(r.float(), h, rtol=2e-2, atol=3e-2)
    hb = r.float()
    ref = hb * torch.rsqrt(hb.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
    torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2)
    # fused [gate | up] projection + SiLU gate
    g = bg.raw(x).finalize_gated(0)
    gu = x.float() @ wg.float().t()
    refg = torch.nn.functional.silu(gu[:, :1024]) * gu[:, 1024:]
    torch.testing.assert_close(g.float(), refg, rtol=3e-2, atol=3e-2)
    # graph: capture one GEMV, replay it several times between eager calls; every replay equals the eager result
    eager = bw.linear(x)
    graph = torch.cuda.CUDAGraph()
    out = torch.empty_like(eager)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        bw.linear(x)  # the capture stream's own workspace gets allocated (and zeroed) outside the capture
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=s):
            out.copy_(bw.linear(x))
    for i in range(4):
        x.add_(0.01 * (i + 1))
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out.float(), bw.linear(x).float(), rtol=1e-2, atol=1e-2)
        torch.cuda.synchronize()
