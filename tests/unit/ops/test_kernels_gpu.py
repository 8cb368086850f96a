"""Numerics of every gfx950 kernel against a plain-PyTorch fp32 reference of the same op
(tolerances as the reference's inference_test_utils: bf16 looser, fp32 tight)."""
import math

import pytest
import torch
import torch.nn.functional as F

from deepspeedsyclsupport_amd.ops import reference as R

pytestmark = pytest.mark.gpu

TOL = {torch.float32: dict(rtol=2e-5, atol=2e-5), torch.bfloat16: dict(rtol=2e-2, atol=2e-2),
       torch.float16: dict(rtol=3e-3, atol=3e-3)}


def ops():
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    return hip_ops()


@pytest.mark.parametrize("n", [1, 1000, 65536 + 3, 1 << 20])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("adamw", [True, False])
def test_adam_flat(n, gdt, adamw):
    torch.manual_seed(0)
    p = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda").abs() * 0.1
    v = torch.rand(n, device="cuda") * 0.1
    g = torch.randn(n, device="cuda").to(gdt)
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    step, lr, b1, b2, eps, wd, gs = 3, 1e-2, 0.9, 0.95, 1e-8, 0.1, 0.5
    ops().adam_flat(p, m, v, g, lp, lr, b1, b2, eps, wd, 1 - b1**step, 1 - b2**step, gs, adamw)
    R.adam_update(pr, mr, vr, g, lr, b1, b2, eps, wd, step, True, adamw, gs)
    torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, mr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v, vr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lp.float(), p.bfloat16().float(), rtol=0, atol=0)


def test_adam_flat_misaligned():
    n = 4099
    base = torch.randn(n + 1, device="cuda")
    p = base[1:]  # 4-byte offset: forces the scalar path
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    g = torch.randn(n, device="cuda")
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    ops().adam_flat(p, m, v, g, None, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, 1.0, True)
    R.adam_update(pr, mr, vr, g, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1)
    torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-6)


def test_adam_multi_and_fused_adam_optimizer():
    from deepspeedsyclsupport_amd.ops.adam import FusedAdam
    torch.manual_seed(1)
    shapes = [(3, 5), (1024, ), (257, 33), (64, 64)] * 10  # > 32 tensors: two launches
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in shapes]
    refs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=0.01)
    ropt = torch.optim.AdamW(refs, lr=1e-2, weight_decay=0.01, eps=1e-8)
    for _ in range(3):
        for p, r in zip(ps, refs):
            g = torch.randn_like(p)
            p.grad, r.grad = g, g.clone()
        opt.step()
        ropt.step()
    for p, r in zip(ps, refs):
        torch.testing.assert_close(p, r, rtol=1e-5, atol=1e-6)


def test_lion_adagrad_lamb():
    torch.manual_seed(2)
    n = 100003
    p, m, g = torch.randn(n, device="cuda"), torch.randn(n, device="cuda") * .1, torch.randn(n, device="cuda")
    pr, mr = p.clone(), m.clone()
    ops().lion_flat(p, m, g, None, 1e-3, 0.9, 0.99, 0.1, 1.0)
    R.lion_update(pr, mr, g, 1e-3, 0.9, 0.99, 0.1)
    torch.testing.assert_close(p, pr)
    torch.testing.assert_close(m, mr)
    s = torch.rand(n, device="cuda")
    sr, pr = s.clone(), p.clone()
    ops().adagrad_flat(p, s, g, None, 1e-2, 1e-10, 0.01, 1.0)
    R.adagrad_update(pr, sr, g, 1e-2, 1e-10, 0.01)
    torch.testing.assert_close(p, pr)
    v = torch.rand(n, device="cuda") * 0.01
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    c = ops().lamb_flat(p, m, v, g, None, 1e-3, 0.9, 0.999, 1e-6, 0.01, 0.1, 0.001, 1.0, 10.0, 0.01)
    trust = R.lamb_update(pr, mr, vr, g, 1e-3, 0.9, 0.999, 1e-6, 0.01, 1, True, 1.0, 10.0, 0.01)
    assert abs(float(c) - trust) < 1e-4 * max(1.0, trust)
    torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-6)


def test_sumsq_multi():
    xs = [torch.randn(n, device="cuda", dtype=dt) for n, dt in [(1000, torch.float32), (77777, torch.bfloat16),
                                                                 (5, torch.float32), (1 << 20, torch.bfloat16)]]
    ref = sum(float(x.float().pow(2).sum()) for x in xs)
    got = float(ops().sumsq_multi(xs))
    assert abs(got - ref) / ref < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H", [64, 1024, 4096, 5120, 8192])
@pytest.mark.parametrize("residual", [False, True])
def test_rms_norm_fwd_bwd(dtype, H, residual):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(3)
    rows = 37
    x = torch.randn(rows, H, device="cuda", dtype=dtype, requires_grad=True)
    r = torch.randn(rows, H, device="cuda", dtype=dtype, requires_grad=True) if residual else None
    w = (1 + 0.1 * torch.randn(H, device="cuda", dtype=dtype)).requires_grad_(True)
    out = DF.rms_norm(x, w, 1e-5, r)
    y = out[0] if residual else out
    xf = x.detach().float().requires_grad_(True)
    rf = r.detach().float().requires_grad_(True) if residual else None
    wf = w.detach().float().requires_grad_(True)
    h = xf + rf if residual else xf
    yr = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    torch.testing.assert_close(y.float(), yr, **TOL[dtype])
    gy = torch.randn_like(yr)
    loss = (y.float() * gy).sum() + ((out[1].float() * gy).sum() if residual else 0)
    loss.backward()
    lr_ = (yr * gy).sum() + ((h * gy).sum() if residual else 0)
    lr_.backward()
    torch.testing.assert_close(x.grad.float(), xf.grad, **TOL[dtype])
    tol = dict(rtol=5e-2, atol=5e-1) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(w.grad.float(), wf.grad, **tol)
    if residual:
        torch.testing.assert_close(r.grad.float(), rf.grad, **TOL[dtype])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H", [768, 1024, 4096, 5120, 8192])
def test_layer_norm_fwd_bwd(dtype, H):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(4)
    x = torch.randn(33, H, device="cuda", dtype=dtype, requires_grad=True)
    g = (1 + 0.1 * torch.randn(H, device="cuda", dtype=dtype)).requires_grad_(True)
    b = (0.1 * torch.randn(H, device="cuda", dtype=dtype)).requires_grad_(True)
    y = DF.layer_norm(x, g, b, 1e-5)
    xf, gf, bf = [t.detach().float().requires_grad_(True) for t in (x, g, b)]
    yr = F.layer_norm(xf, (H, ), gf, bf, 1e-5)
    torch.testing.assert_close(y.float(), yr, **TOL[dtype])
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xf.grad, **TOL[dtype])
    tol = dict(rtol=5e-2, atol=5e-1) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(g.grad.float(), gf.grad, **tol)
    torch.testing.assert_close(b.grad.float(), bf.grad, **tol)


@pytest.mark.parametrize("H", [1032, 2048, 5120])
@pytest.mark.parametrize("kind", ["rms", "ln"])
def test_norm_backward_many_rows(kind, H):
    """More rows than persistent blocks (every block walks several rows, the column partials of all blocks are
    summed) and a width that is not a multiple of the block's 2048-element step."""
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(6)
    rows = 2100
    x = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = (1 + 0.1 * torch.randn(H, device="cuda", dtype=torch.bfloat16)).requires_grad_(True)
    b = (0.1 * torch.randn(H, device="cuda", dtype=torch.bfloat16)).requires_grad_(True)
    xf, gf, bf = [t.detach().float().requires_grad_(True) for t in (x, g, b)]
    if kind == "rms":
        y = DF.rms_norm(x, g, 1e-5)
        yr = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * gf
    else:
        y = DF.layer_norm(x, g, b, 1e-5)
        yr = F.layer_norm(xf, (H, ), gf, bf, 1e-5)
    gy = torch.randn_like(yr).bfloat16().float()
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xf.grad, **TOL[torch.bfloat16])
    # column sums over 2100 rows of bf16-rounded products: compare against the fp32 sum with a relative bound
    scale = float(gf.grad.abs().max())
    assert float((g.grad.float() - gf.grad).abs().max()) <= 2e-2 * scale
    if kind == "ln":
        assert float((b.grad.float() - bf.grad).abs().max()) <= 2e-2 * float(bf.grad.abs().max())


@pytest.mark.parametrize("act", ["silu", "gelu", "gelu_tanh", "relu"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gated_act(act, dtype):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(5)
    gu = torch.randn(19, 2 * 1376, device="cuda", dtype=dtype, requires_grad=True)
    y = DF.gated_activation(gu, act)
    gf = gu.detach().float().requires_grad_(True)
    a, u = gf.chunk(2, -1)
    fn = {"silu": F.silu, "gelu": F.gelu, "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"), "relu": F.relu}[act]
    yr = fn(a) * u
    torch.testing.assert_close(y.float(), yr, **TOL[dtype])
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(gu.grad.float(), gf.grad, **TOL[dtype])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_bias_act(dtype):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    x = torch.randn(13, 3072, device="cuda", dtype=dtype, requires_grad=True)
    b = torch.randn(3072, device="cuda", dtype=dtype, requires_grad=True)
    y = DF.bias_activation(x, b, "gelu_tanh")
    xf, bf = x.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    yr = F.gelu(xf + bf, approximate="tanh")
    torch.testing.assert_close(y.float(), yr, **TOL[dtype])
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xf.grad, **TOL[dtype])


@pytest.mark.parametrize("token_major", [False, True])
@pytest.mark.parametrize("hq,hk", [(8, 8), (8, 2)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_qkv_rope_split(hq, hk, dtype, token_major):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(6)
    B, S, D = 2, 33, 128
    cos, sin = R.rope_tables(128, D, device="cuda")
    qkv = torch.randn(B, S, hq + 2 * hk, D, device="cuda", dtype=dtype, requires_grad=True)
    q, k, v = DF.qkv_rope_split(qkv, cos, sin, hq, hk, token_major=token_major)
    assert q.transpose(1, 2).is_contiguous() == token_major
    qf = qkv.detach().float().requires_grad_(True)
    qq, kk, vv = qf.split([hq, hk, hk], dim=2)
    pos = torch.arange(S, device="cuda")
    qr = R.apply_rope_half(qq, cos, sin, pos).transpose(1, 2)
    kr = R.apply_rope_half(kk, cos, sin, pos).transpose(1, 2)
    vr = vv.transpose(1, 2)
    for a, b in ((q, qr), (k, kr), (v, vr)):
        torch.testing.assert_close(a.float(), b, **TOL[dtype])
    gs = [torch.randn_like(t) for t in (qr, kr, vr)]
    sum((a.float() * g).sum() for a, g in zip((q, k, v), gs)).backward()
    sum((a * g).sum() for a, g in zip((qr, kr, vr), gs)).backward()
    torch.testing.assert_close(qkv.grad.float(), qf.grad, **TOL[dtype])


@pytest.mark.parametrize("interleaved", [False, True])
def test_rope_inplace(interleaved):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    B, S, H, D = 2, 17, 4, 64
    cos, sin = R.rope_tables(64, D, device="cuda")
    x = torch.randn(B, S, H, D, device="cuda")
    ref = DF.apply_rotary_pos_emb(x.clone().cpu(), cos.cpu(), sin.cpu(), interleaved=interleaved)
    got = DF.apply_rotary_pos_emb(x.clone(), cos, sin, interleaved=interleaved)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-5, atol=1e-5)
    back = DF.apply_rotary_pos_emb(got.clone(), cos, sin, interleaved=interleaved, inverse=True)
    torch.testing.assert_close(back, x, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("V", [32000, 50257, 1000])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cross_entropy(V, dtype):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(7)
    N = 67
    logits = (3 * torch.randn(N, V, device="cuda")).to(dtype).requires_grad_(True)
    labels = torch.randint(0, V, (N, ), device="cuda")
    labels[3] = -100
    loss = DF.cross_entropy(logits, labels, inplace_backward=False)
    lf = logits.detach().float().requires_grad_(True)
    lr_ = F.cross_entropy(lf, labels, ignore_index=-100)
    torch.testing.assert_close(loss.float(), lr_, rtol=1e-4, atol=1e-4)
    loss.backward()
    lr_.backward()
    torch.testing.assert_close(logits.grad.float(), lf.grad, **TOL[dtype])


# ------------------------------------------------------------------------------------------------ inference kernels
def _paged_setup(B, Hk, D, BS, lens, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    maxb = max((L + BS - 1) // BS for L in lens)
    nb = B * maxb + 3
    kc = torch.randn(nb, Hk, BS, D, device="cuda", generator=g).bfloat16()
    vc = torch.randn(nb, Hk, BS, D, device="cuda", generator=g).bfloat16()
    perm = torch.randperm(nb, device="cuda", generator=g)[:B * maxb].to(torch.int32).view(B, maxb)
    return kc, vc, perm.contiguous(), maxb


def _paged_ref(q, kc, vc, bt, lens, scale, alibi=None, window=0):
    B, Hq, D = q.shape
    Hk, BS = kc.shape[1], kc.shape[2]
    out = torch.empty(B, Hq, D, device="cuda")
    for b in range(B):
        L = lens[b]
        nblk = (L + BS - 1) // BS
        ids = bt[b, :nblk].long()
        k = kc[ids].float().transpose(0, 1).reshape(Hk, -1, D)[:, :L]
        v = vc[ids].float().transpose(0, 1).reshape(Hk, -1, D)[:, :L]
        k, v = k.repeat_interleave(Hq // Hk, 0), v.repeat_interleave(Hq // Hk, 0)
        s = torch.einsum("hd,htd->ht", q[b].float(), k) * scale
        if alibi is not None:
            s = s + alibi[:, None] * (torch.arange(L, device="cuda") - (L - 1)).float()[None]
        if window:
            s[:, :max(0, L - window)] = float("-inf")
        out[b] = torch.einsum("ht,htd->hd", s.softmax(-1), v)
    return out


@pytest.mark.parametrize("D", [64, 80, 96, 128, 256])
@pytest.mark.parametrize("hq,hk", [(8, 8), (32, 8), (8, 1)])
@pytest.mark.parametrize("lens", [[1, 7, 64], [300, 2049, 5000]])
def test_paged_decode(D, hq, hk, lens):
    B, BS = len(lens), 64
    kc, vc, bt, maxb = _paged_setup(B, hk, D, BS, lens)
    q = torch.randn(B, hq, D, device="cuda").bfloat16()
    sl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    out = ops().paged_decode(q, kc, vc, bt, sl, max(lens), scale, None, 0)
    ref = _paged_ref(q, kc, vc, bt, lens, scale)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


def test_paged_decode_alibi_window_and_capacity():
    B, hq, hk, D, BS = 3, 8, 8, 128, 16
    lens = [5, 40, 100]
    kc, vc, bt, maxb = _paged_setup(B, hk, D, BS, lens, seed=3)
    q = torch.randn(B, hq, D, device="cuda").bfloat16()
    sl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    from deepspeedsyclsupport_amd.inference.model_implementations.transformer import alibi_slopes
    al = alibi_slopes(hq).cuda()
    # max_len = full block-table capacity (the HIP-graph decode path): empty splits must not perturb the result
    out = ops().paged_decode(q, kc, vc, bt, sl, maxb * BS, 0.1, al, 32)
    ref = _paged_ref(q, kc, vc, bt, lens, 0.1, al, 32)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


def test_kv_append():
    B, n, hk, D, BS = 3, 5, 4, 128, 16
    kc, vc, bt, maxb = _paged_setup(B, hk, D, BS, [64, 64, 64])
    k = torch.randn(B, n, hk, D, device="cuda").bfloat16()
    v = torch.randn(B, n, hk, D, device="cuda").bfloat16()
    start = torch.tensor([0, 14, 40], dtype=torch.int32, device="cuda")
    kr, vr = kc.clone(), vc.clone()
    ops().kv_append(k, v, kc, vc, bt, start)
    for b in range(B):
        for j in range(n):
            t = int(start[b]) + j
            blk = int(bt[b, t // BS])
            kr[blk, :, t % BS] = k[b, j]
            vr[blk, :, t % BS] = v[b, j]
    assert torch.equal(kc, kr) and torch.equal(vc, vr)


@pytest.mark.parametrize("bits", [8, 4])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_quantize_roundtrip(bits, sym, dtype):
    from deepspeedsyclsupport_amd.ops.quantizer.quantizer import _ref_dequantize, _ref_quantize
    torch.manual_seed(0)
    gs = 128
    x = (torch.randn(64 * gs, device="cuda") * 3).to(dtype)
    q, s, z = ops().quantize(x, gs, bits, not sym, False, 0)
    qr, sr, zr = _ref_quantize(x.cpu(), gs, bits, not sym)
    torch.testing.assert_close(s.cpu(), sr, rtol=1e-5, atol=1e-7)
    d = ops().dequantize(q, s, z if not sym else None, x.numel(), gs, bits, torch.float32)
    dr = _ref_dequantize(qr, sr, zr, x.numel(), gs, bits, torch.float32)
    # kernel and reference may round exact .5 ties differently: allow one quantisation step
    step = s.repeat_interleave(gs).cpu()
    assert ((d.cpu() - dr).abs() <= step * 1.01 + 1e-6).all()
    assert ((x.float() - d).abs() <= s.repeat_interleave(gs) * 0.51 + 1e-5).all()


def test_dequant_reduce():
    from deepspeedsyclsupport_amd.ops.quantizer import quantize
    torch.manual_seed(0)
    gs, n, k = 256, 256 * 32, 4
    xs = [torch.randn(n, device="cuda") for _ in range(k)]
    qts = [quantize(x, gs, 8) for x in xs]
    q = torch.cat([t.data for t in qts])
    s = torch.cat([t.scales for t in qts])
    out = ops().dequant_reduce(q, s, k, gs, 0.25, torch.float32)
    ref = sum(x for x in xs) * 0.25
    torch.testing.assert_close(out, ref, rtol=0, atol=k * 0.25 * float(s.max()) * 0.51)


@pytest.fixture(params=["mfma", "valu", "auto"])
def skinny_path(request):
    ops().skinny_set_path({"auto": 0, "valu": 1, "mfma": 2}[request.param])
    yield request.param
    ops().skinny_set_path(0)


@pytest.mark.parametrize("M", [1, 2, 3, 5, 8, 12, 16])
@pytest.mark.parametrize("N,K", [(4096, 4096), (333, 11008), (7, 64), (100, 256), (50, 768)])
def test_skinny_gemm_plain(M, N, K, skinny_path):
    if M > 8 and (K % 256 or skinny_path == "valu"):
        pytest.skip("rows > 8 need the MFMA kernel (K % 256 == 0)")
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    add = torch.randn(M, N, device="cuda").bfloat16()
    y = ops().skinny_gemm(x, w, b, add, 0, False, 0, None, None, 0.0, None)
    ref = x.float() @ w.float().t() + b.float() + add.float()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M", [1, 4, 8, 16])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("K", [4096, 8192])
def test_skinny_gemm_rmsnorm(M, with_res, K, skinny_path):
    if M > 8 and skinny_path == "valu":
        pytest.skip("rows > 8 need the MFMA kernel")
    torch.manual_seed(1)
    N, eps = 1000, 1e-5
    x = torch.randn(M, K, device="cuda").bfloat16()
    r = torch.randn(M, K, device="cuda").bfloat16() if with_res else None
    nw = (1 + 0.1 * torch.randn(K, device="cuda")).bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    res_out = torch.empty_like(x)
    y = ops().skinny_gemm(x, w, None, None, 1, False, 0, r, nw, eps, res_out)
    y2 = ops().skinny_gemm(x, w, None, None, 1, False, 0, r, nw, eps, None)  # LM-head form: no residual output
    torch.testing.assert_close(y2, y, rtol=0, atol=0)
    h = (x.float() + (r.float() if with_res else 0)).bfloat16().float()
    normed, _ = R.rms_norm(h, nw.float(), eps)
    torch.testing.assert_close(y.float(), normed @ w.float().t(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(res_out.float(), h.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("act", ["silu", "gelu", "relu"])
@pytest.mark.parametrize("M", [1, 3, 8, 16])
def test_skinny_gemm_gated(act, M, skinny_path):
    if M > 8 and skinny_path == "valu":
        pytest.skip("rows > 8 need the MFMA kernel")
    from deepspeedsyclsupport_amd.ops.transformer.functional import ACT_CODES
    torch.manual_seed(2)
    I, K = 1376, 4096
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(2 * I, K, device="cuda") * 0.02).bfloat16()
    b = torch.randn(2 * I, device="cuda").bfloat16()
    y = ops().skinny_gemm(x, w, b, None, 0, True, ACT_CODES[act], None, None, 0.0, None)
    gu = (x.float() @ w.float().t() + b.float()).bfloat16().float()
    ref = R.gated_act(gu, ACT_CODES[act])
    assert y.shape == (M, I)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("rot,interleaved", [(128, False), (32, False), (64, True), (0, False)])
def test_qkv_rope_append(rot, interleaved):
    torch.manual_seed(3)
    B, n, hq, hk, D, BS = 2, 5, 8, 2, 128, 16
    kc, vc, bt, maxb = _paged_setup(B, hk, D, BS, [64, 64])
    qkv = torch.randn(B * n, (hq + 2 * hk) * D, device="cuda").bfloat16()
    start = torch.tensor([3, 20], dtype=torch.int32, device="cuda")
    pos = (start[:, None] + torch.arange(n, device="cuda", dtype=torch.int32)[None]).reshape(-1).contiguous()
    cos, sin = R.rope_tables(256, max(rot, 2), device="cuda")
    kr, vr = kc.clone(), vc.clone()
    q, k, v = ops().qkv_rope_append(qkv, cos if rot else None, sin if rot else None, pos, kc, vc, bt, start, n, hq,
                                    hk, rot, interleaved, True)
    x = qkv.view(B, n, hq + 2 * hk, D).float()
    qr, krr, vrr = x[:, :, :hq].clone(), x[:, :, hq:hq + hk].clone(), x[:, :, hq + hk:].clone()
    p = pos.view(B, n).long()
    if rot:
        def rope(t):
            if interleaved:
                c, s = cos[p][:, :, None, :], sin[p][:, :, None, :]
                a, b_ = t[..., 0:rot:2].clone(), t[..., 1:rot:2].clone()
                t[..., 0:rot:2], t[..., 1:rot:2] = a * c - b_ * s, b_ * c + a * s
                return t
            return R.apply_rope_half(t, cos, sin, p)
        qr, krr = rope(qr), rope(krr)
    torch.testing.assert_close(q.float().view(B, n, hq, D), qr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(k.float().view(B, n, hk, D), krr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(v.float().view(B, n, hk, D), vrr, rtol=0, atol=0)
    for b in range(B):
        for j in range(n):
            t = int(start[b]) + j
            blk = int(bt[b, t // BS])
            kr[blk, :, t % BS] = k.view(B, n, hk, D)[b, j]
            vr[blk, :, t % BS] = v.view(B, n, hk, D)[b, j]
    assert torch.equal(kc, kr) and torch.equal(vc, vr)


def _unpack_mask(packed, shape):
    bits = (packed.long().unsqueeze(-1) >> torch.arange(8, device=packed.device)) & 1
    return bits.reshape(shape).bool()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("p", [0.1, 0.5])
def test_fused_dropout(dt, p):
    """residual + dropout(x + bias) vs the same math in fp32 with the kernel's own mask; the mask's keep rate; the
    backward regenerates the identical mask from the seed (no stored mask)."""
    torch.manual_seed(0)
    rows, C = 1000, 1024
    x = torch.randn(rows, C, device="cuda").to(dt)
    b = torch.randn(C, device="cuda").to(dt)
    r = torch.randn(rows, C, device="cuda").to(dt)
    y, packed = ops().dropout_fwd(x, b, r, p, 1234, 0, True)
    keep = _unpack_mask(packed, (rows, C))
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 0.01, rate
    ref = r.float() + torch.where(keep, (x.float() + b.float()) / (1 - p), torch.zeros_like(x.float()))
    torch.testing.assert_close(y.float(), ref, **TOL[dt])
    dy = torch.randn(rows, C, device="cuda").to(dt)
    dx = ops().dropout_bwd(dy, p, 1234, 0)
    ref_dx = torch.where(keep, dy.float() / (1 - p), torch.zeros_like(dy.float()))
    torch.testing.assert_close(dx.float(), ref_dx, **TOL[dt])
    # a different seed gives a different mask; same seed the same one
    _, p2 = ops().dropout_fwd(x, None, None, p, 1235, 0, True)
    _, p3 = ops().dropout_fwd(x, None, None, p, 1234, 0, True)
    assert not torch.equal(p2, packed) and torch.equal(p3, packed)


def test_dropout_autograd_and_checkpoint_replay():
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(1)
    # positive x and b: x + b is never 0, so y0 != 0 identifies the kept elements
    x = (torch.rand(64, 256, device="cuda") + 0.1).bfloat16().requires_grad_(True)
    b = (torch.rand(256, device="cuda") + 0.1).bfloat16().requires_grad_(True)
    r = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    torch.manual_seed(7)
    y0 = DF.dropout(x, 0.2, True, bias=b)
    keep = y0 != 0
    torch.manual_seed(7)
    y = DF.dropout(x, 0.2, True, bias=b, residual=r)
    torch.testing.assert_close(y.float(), (r.float() + y0.float()), rtol=2e-2, atol=2e-2)
    y.float().sum().backward()
    torch.testing.assert_close(x.grad.float(), keep.float() / 0.8, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(b.grad.float(), (keep.float() / 0.8).sum(0), rtol=2e-2, atol=2e-1)
    assert torch.equal(r.grad, torch.ones_like(r))
    torch.manual_seed(7)
    y2 = torch.utils.checkpoint.checkpoint(lambda t: DF.dropout(t, 0.2, True, bias=b, residual=r), x,
                                           use_reentrant=False)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_spatial_nhwc_bias_add(dt):
    from deepspeedsyclsupport_amd.ops import spatial
    torch.manual_seed(2)
    x = torch.randn(2, 320, 16, 16, device="cuda").to(dt).to(memory_format=torch.channels_last)
    o = torch.randn(2, 320, 16, 16, device="cuda").to(dt).to(memory_format=torch.channels_last)
    b, ob = torch.randn(320, device="cuda").to(dt), torch.randn(320, device="cuda").to(dt)
    bb, obb = b.view(1, -1, 1, 1).float(), ob.view(1, -1, 1, 1).float()
    torch.testing.assert_close(spatial.nhwc_bias_add(x, b).float(), x.float() + bb, **TOL[dt])
    torch.testing.assert_close(spatial.nhwc_bias_add_add(x, b, o).float(), x.float() + bb + o.float(), **TOL[dt])
    torch.testing.assert_close(spatial.nhwc_bias_add_bias_add(x, b, o, ob).float(),
                               x.float() + bb + o.float() + obb, **TOL[dt])


@pytest.mark.parametrize("M", [1, 2, 4, 5, 8, 16])
@pytest.mark.parametrize("N,K,gs", [(1, 64, 64), (13, 4096, 64), (4096, 11008, 64), (1000, 14336, 128), (300, 57344, 64),
                                    (77, 320, 64), (50, 4160, 64), (129, 2048, 512), (64, 1024, 1024)])
@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("path", ["valu", "mfma"])
def test_skinny_int8_gemv(M, N, K, gs, bias, path):
    """Weight-only int8 decode GEMV (fused group dequant) vs an fp32 GEMM on the dequantised weight: the VALU stream
    over the row-major weight (<= 8 rows) and the MFMA stream over the pre-shuffled weight (<= 16 rows)."""
    from deepspeedsyclsupport_amd.ops.int8_gemv import preshuffle
    from deepspeedsyclsupport_amd.ops.quantizer import dequantize, quantize
    torch.manual_seed(N + K)
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    qt = quantize(w, group_size=gs, bits=8, symmetric=True)
    x = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda").bfloat16() if bias else None
    if path == "valu":
        if M > 8:
            pytest.skip("VALU stream is for <= 8 rows")
        y = ops().skinny_i8(x, qt.data, qt.scales, b, N, gs)
    else:
        qsh, ssh = preshuffle(qt.data.view(N, K), qt.scales, gs)
        y = ops().skinny_i8_sh(x, qsh, ssh, b, N, gs)
    ref = x.float() @ dequantize(qt, torch.float32).t()
    if bias:
        ref = ref + b.float()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * max(1.0, ref.abs().max().item()))


def test_skinny_int8_mfma_workspace_reuse_and_graph():
    """The MFMA path's split-K workspace re-zeroes itself: repeated calls, interleaved shapes and a HIP-graph replay
    all give the first call's result; Int8Weight.linear routes decode sizes to it and prefill to dequant + GEMM."""
    from deepspeedsyclsupport_amd.ops.int8_gemv import Int8Weight
    torch.manual_seed(3)
    mats = []
    for N, K in ((4096, 4096), (11008, 4096), (333, 8192)):
        wt = Int8Weight((torch.randn(N, K, device="cuda") * 0.02).bfloat16(), 64)
        mats.append((wt, torch.randn(8, K, device="cuda").bfloat16()))
    first = [wt.linear(x) for wt, x in mats]
    for wt, x in mats:  # native bf16 dequant from the shuffled layout == host un-shuffle + dequant
        torch.testing.assert_close(wt.materialize().float(), wt.materialize(torch.float32), rtol=1e-2, atol=1e-4)
    for wt, x in mats:
        ref = x.float() @ wt.materialize(torch.float32).t()
        torch.testing.assert_close(first[mats.index((wt, x))].float(), ref, rtol=2e-2, atol=2e-2)
    for _ in range(3):
        for (wt, x), y0 in zip(mats, first):
            torch.testing.assert_close(wt.linear(x), y0, rtol=1e-2, atol=1e-2)
    wt, x = mats[1]
    xp = torch.randn(40, x.shape[1], device="cuda").bfloat16()  # prefill-sized: dequant + library GEMM
    torch.testing.assert_close(wt.linear(xp).float(), xp.float() @ wt.materialize(torch.float32).t(), rtol=2e-2,
                               atol=2e-2)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        wt.linear(x)  # workspace for this stream exists before capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        yg = wt.linear(x)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(yg, first[1], rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("H", [14336, 16384])
@pytest.mark.parametrize("res", [False, True])
def test_wide_norm_forward(H, res):
    """Forward LayerNorm / RMSNorm on BLOOM-176B-wide rows (wide NV buckets) vs fp32 references."""
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(H)
    x = torch.randn(5, H, device="cuda").bfloat16()
    r = torch.randn(5, H, device="cuda").bfloat16() if res else None
    g = torch.randn(H, device="cuda").bfloat16()
    b = torch.randn(H, device="cuda").bfloat16()
    h = x.float() + (r.float() if res else 0)
    with torch.no_grad():
        y = DF.layer_norm(x, g, b, 1e-5, r)
        y = y[0] if res else y
        yr = DF.rms_norm(x, g, 1e-6, r)
        yr = yr[0] if res else yr
    ref = F.layer_norm(h, (H, ), g.float(), b.float(), 1e-5)
    ref_r = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(yr.float(), ref_r, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("rows", [1, 16, 256, 300])
@pytest.mark.parametrize("H", [1024, 4096, 5120, 14336])
@pytest.mark.parametrize("res", [False, True])
def test_norm_forward_few_and_many_rows(rows, H, res):
    """Up to 256 rows a block owns each row (decode-sized inputs), beyond that a wave does: both against fp32, with
    the saved statistics checked through the backward of the training path."""
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(rows * 7 + H)
    x = torch.randn(rows, H, device="cuda").bfloat16()
    r = torch.randn(rows, H, device="cuda").bfloat16() if res else None
    g = (1 + 0.1 * torch.randn(H, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(H, device="cuda")).bfloat16()
    h = x.float() + (r.float() if res else 0)
    with torch.no_grad():
        y = DF.layer_norm(x, g, b, 1e-5, r)
        yr = DF.rms_norm(x, g, 1e-6, r)
    if res:
        torch.testing.assert_close(y[1].float(), h.bfloat16().float(), rtol=0, atol=0)
        torch.testing.assert_close(yr[1].float(), h.bfloat16().float(), rtol=0, atol=0)
        y, yr = y[0], yr[0]
    ref = F.layer_norm(h, (H, ), g.float(), b.float(), 1e-5)
    ref_r = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(yr.float(), ref_r, rtol=2e-2, atol=2e-2)
    if H <= 8192 and not res:  # the backward kernels (hidden <= 8192) consume the forward's mean / rstd
        xg = x.clone().requires_grad_(True)
        xf = x.float().requires_grad_(True)
        gy = torch.randn(rows, H, device="cuda")
        (DF.layer_norm(xg, g, b, 1e-5).float() * gy).sum().backward()
        (F.layer_norm(xf, (H, ), g.float(), b.float(), 1e-5) * gy).sum().backward()
        torch.testing.assert_close(xg.grad.float(), xf.grad, rtol=5e-2, atol=5e-2)
