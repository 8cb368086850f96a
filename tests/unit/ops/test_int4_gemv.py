"""Weight-only int4: packed operand layout (CPU), fused-dequant MFMA stream and the packed-layout dequantiser (GPU)
against fp32 math on the dequantised weight (reference `inference/v2/kernels/cutlass_ops/mixed_gemm` with num_bits=4,
`op_builder/inference_cutlass_builder.py`; no reference-produced fixture exists, byte parity unpinned)."""
import pytest
import torch

from deepspeedsyclsupport_amd.ops import int4_gemv as i4


@pytest.mark.parametrize("N,K,gs", [(40, 256, 64), (16, 128, 32), (33, 512, 128), (64, 512, 256), (7, 384, 384)])
def test_pack_roundtrip_and_nibble_order(N, K, gs):
    torch.manual_seed(0)
    q = torch.randint(-8, 8, (N, K), dtype=torch.int8)
    s = torch.rand(N * K // gs) + 0.1
    q4, s4 = i4.pack_int4_operands(q, s, gs)
    assert q4.shape == ((N + 15) // 16, K // 128, 64, 16) and q4.dtype == torch.int8
    q2, s2 = i4.unpack_int4_operands(q4, s4, N)
    assert torch.equal(q, q2) and torch.equal(s, s2)
    # the kernel's extraction: register t of word i = nibbles (t, t + 4) = operand elements (2t, 2t + 1)
    words = q4.contiguous().view(torch.int32).reshape(-1, K // 128, 64, 4)
    nb, kq, lane, i = 0, K // 128 - 1, 37, 2
    w = int(words[nb, kq, lane, i]) & 0xFFFFFFFF
    elems = []
    for t in range(4):
        reg = (w >> (4 * t)) & 0x000F000F
        elems += [reg & 0xFFFF, reg >> 16]
    r, g = lane & 15, lane >> 4
    if 16 * nb + r < N:
        assert elems == [int(q[16 * nb + r, 128 * kq + 32 * i + 8 * g + j]) + 8 for j in range(8)]


def test_bf16_offset_encoding_is_exact():
    """0x4300 | u is the bf16 number 128 + u for every nibble value."""
    u = torch.arange(16, dtype=torch.int16)
    assert torch.equal((u | 0x4300).view(torch.bfloat16).float(), 128.0 + u.float())


def test_int4_weight_cpu_linear_and_group_rules():
    torch.manual_seed(1)
    w = torch.randn(48, 256)
    iw = i4.Int4Weight(w, 64)
    d = iw.materialize(torch.float32)
    assert (d - w).abs().max() <= w.abs().max() / 7 * 0.51 + 1e-6
    x = torch.randn(3, 256)
    torch.testing.assert_close(iw.linear(x), x @ d.t())
    assert i4.Int4Weight.supported(w, 4, 64) and i4.Int4Weight.supported(w, 4, 128)
    assert not i4.Int4Weight.supported(w, 8, 64) and not i4.Int4Weight.supported(torch.randn(8, 192), 4, 64)
    assert iw.nbytes() == 48 * 256 // 2 + 48 * 4 * 4


def test_builder_reports_native_int4():
    from deepspeedsyclsupport_amd.ops.op_builder import InferenceCutlassBuilder
    b = InferenceCutlassBuilder()
    assert b.is_compatible(num_bits=4) == b.is_compatible(num_bits=8)


def test_mixed_gemm_int4_cpu():
    """reference call contract: weights [in, out // 2] packed per output channel, scales [out]."""
    from deepspeedsyclsupport_amd.ops import cutlass_ops as C
    torch.manual_seed(2)
    K, N = 256, 24
    q = torch.randint(-8, 8, (K, N), dtype=torch.int8)
    scales = torch.rand(N) * 0.1 + 0.01
    x = torch.randn(5, K).bfloat16()
    out = torch.empty(5, N, dtype=torch.bfloat16)
    C.MixedGEMM(torch.bfloat16, "identity", 4)(out, x, C.pack_int4(q), scales)
    ref = x.float() @ (q.float() * scales[None])
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K,gs", [(4096, 4096, 128), (1000, 512, 64), (72, 1024, 32), (256, 11008 // 128 * 128, 256),
                                    (130, 256, 256)])
@pytest.mark.parametrize("bias", [False, True])
def test_skinny_int4_gemv(M, N, K, gs, bias):
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(M + N)
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    iw = i4.Int4Weight(w, gs)
    x = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda").bfloat16() if bias else None
    q, s = i4.unpack_int4_operands(iw.q4.cpu(), iw.s4.cpu(), N)
    wd = (q.float().reshape(N, K // gs, gs) * s.reshape(N, -1, 1)).reshape(N, K).cuda()
    ref = x.float() @ wd.t() + (b.float() if bias else 0.0)
    y = hip_ops().skinny_i4(x, iw.q4, iw.s4, b, N, gs)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item() + 1e-3)
    # packed-layout dequantiser (prefill path) is exact up to bf16 rounding of scale * q
    torch.testing.assert_close(iw.materialize().float(), wd.bfloat16().float(), rtol=0, atol=0)
    assert iw.linear(x, b).shape == (M, N)


@pytest.mark.gpu
def test_skinny_int4_workspace_reuse_and_graph():
    """Back-to-back calls with different N share the fp32 workspace (re-zeroed by the finalize kernel), and the op
    replays inside a HIP graph with eager work in between."""
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    torch.manual_seed(0)
    ws = [i4.Int4Weight((torch.randn(n, 512, device="cuda") * 0.05).bfloat16(), 128) for n in (640, 100, 2048)]
    x = torch.randn(4, 512, device="cuda").bfloat16()
    eager = [w.linear(x).clone() for w in ws]
    for w, e in zip(ws, eager):
        torch.testing.assert_close(w.linear(x), e, rtol=0, atol=0)
    static_x = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            ws[0].linear(static_x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = ws[0].linear(static_x)
    for it in range(3):
        xn = torch.randn(4, 512, device="cuda").bfloat16()
        static_x.copy_(xn)
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out, ws[0].linear(xn), rtol=0, atol=0)
        ws[1].linear(xn)  # eager work between replays


@pytest.mark.gpu
def test_int4_decode_follows_bf16_engine():
    """Weight-only int4 engine: decode steps take the packed MFMA stream, prefill the dequantise + GEMM path; the
    last-token logits follow the bf16 engine within int4 quantisation noise."""
    import copy

    import deepspeedsyclsupport_amd as ds
    from tests.unit.inference.test_inference import _ids, tiny
    m = tiny("llama", H=256).eval()
    ids = _ids(B=2, S=12).cuda()
    e16 = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True)
    e4 = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True,
                           quant={"enabled": True, "weight": {"num_bits": 4, "q_groups": 1}})
    lay = e4.module.layers[0]
    assert lay.quant and all(isinstance(q.i8, i4.Int4Weight) for q in lay.quant.values())
    g16 = e16.generate(ids, max_new_tokens=6)
    l16 = e16(g16[:, :-1]).logits[:, -1].float()
    l4 = e4(g16[:, :-1]).logits[:, -1].float()
    assert (l4 - l16).abs().max().item() < 0.35 * l16.abs().max().item() + 0.1
    assert e4.generate(ids, max_new_tokens=6).shape == g16.shape


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("M,N,K", [(1, 4096, 512), (5, 1000, 256), (16, 14336, 256), (3, 72, 128)])
def test_fused_finalize_consumers(bits, M, N, K):
    """The stream without its finalize pass + (residual add + RMSNorm | gated activation | plain) consumers equal
    the finalized GEMV followed by the separate ops, and leave the workspace zero for the next call."""
    from deepspeedsyclsupport_amd.ops import reference
    from deepspeedsyclsupport_amd.ops.int8_gemv import Int8Weight
    from deepspeedsyclsupport_amd.ops.transformer.functional import ACT_CODES
    torch.manual_seed(bits + M)
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    W = i4.Int4Weight(w, 128) if bits == 4 else Int8Weight(w, 64)
    x = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()
    lnw = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16()
    y = W.linear(x).float()                       # no bias: the workspace sums
    # plain
    torch.testing.assert_close(W.raw(x, b).finalize().float(), (y + b.float()).bfloat16().float(), rtol=1e-2, atol=1e-2)
    # residual + RMSNorm
    out, new_res = W.raw(x, b).finalize_rms(res, lnw, 1e-5)
    r_ref = (y + b.float() + res.float()).bfloat16()
    torch.testing.assert_close(new_res.float(), r_ref.float(), rtol=1e-2, atol=2e-2)
    rf = new_res.float()
    n_ref = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + 1e-5) * lnw.float()
    torch.testing.assert_close(out.float(), n_ref, rtol=2e-2, atol=2e-2)
    out2, _ = W.raw(x).finalize_rms(None, lnw, 1e-5)  # no bias, no residual
    n2 = y * torch.rsqrt(y.bfloat16().float().pow(2).mean(-1, keepdim=True) + 1e-5) * lnw.float()
    torch.testing.assert_close(out2.float(), n2, rtol=2e-2, atol=2e-2)
    # gated activation
    if N % 2 == 0:
        for act in ("silu", "gelu"):
            g = W.raw(x, b).finalize_gated(ACT_CODES[act])
            yy = y + b.float()
            ref = reference.ACTS[ACT_CODES[act]](yy[:, :N // 2]) * yy[:, N // 2:]
            torch.testing.assert_close(g.float(), ref, rtol=2e-2, atol=2e-2)
    # the workspace is zero again: a plain call still matches
    torch.testing.assert_close(W.linear(x).float(), y, rtol=0, atol=0)
    p = W.raw(x)
    p.finalize()
    with pytest.raises(RuntimeError):
        p.finalize()
