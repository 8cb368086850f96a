"""gfx950 MoE routing / grouped-GEMM / ragged-gather kernels vs plain-PyTorch fp32 references
(reference tests: `tests/unit/inference/v2/kernels/ragged_ops/test_top_k_gating.py`, `test_moe_scatter.py`,
`test_moe_gather.py`, `kernels/cutlass_ops/test_moe_gemm.py`, `ragged_ops/test_ragged_embed.py`,
`test_logits_gather.py`)."""
import pytest
import torch
import torch.nn.functional as F

from deepspeedsyclsupport_amd.ops import moe_ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (37, 8, 2), (300, 64, 6), (129, 256, 8), (5, 3, 3)])
@pytest.mark.parametrize("renorm", [False, True])
def test_topk_gating(T, E, k, renorm):
    torch.manual_seed(T + E)
    # distinct values per row (k/16 is exact in bf16 for k < 256) so the top-k order has no ties
    logits = (torch.stack([torch.randperm(E) for _ in range(T)]).float() / 16).bfloat16().cuda()
    scores, experts, slots, counts = moe_ops.topk_gating(logits, k, renorm)
    w_ref, e_ref, c_ref = moe_ops.topk_gating_reference(logits, k, renorm)
    assert torch.equal(experts.long(), e_ref)
    torch.testing.assert_close(scores, w_ref, rtol=1e-5, atol=1e-6)
    assert torch.equal(counts.long(), c_ref)
    # slots: within each expert a permutation of 0..count-1
    for e in range(E):
        s = slots[experts == e].sort().values
        assert torch.equal(s.cpu(), torch.arange(int(c_ref[e]), dtype=torch.int32))


@pytest.mark.parametrize("T,H,E,k", [(64, 256, 8, 2), (333, 512, 16, 4)])
def test_scatter_gather_roundtrip(T, H, E, k):
    torch.manual_seed(1)
    x = torch.randn(T, H, device="cuda").bfloat16()
    scores, experts, slots, counts = moe_ops.topk_gating(torch.randn(T, E, device="cuda"), k)
    xs, rows, cumsum = moe_ops.moe_scatter(x, experts, slots, counts)
    assert torch.equal(cumsum, counts.long().cumsum(0))
    # rows of expert e are the contiguous range [cumsum[e]-count[e], cumsum[e])
    start = cumsum - counts.long()
    for t in (0, T // 2, T - 1):
        for j in range(k):
            r = int(rows[t, j])
            e = int(experts[t, j])
            assert int(start[e]) <= r < int(cumsum[e])
            assert torch.equal(xs[r], x[t])
    out = moe_ops.moe_gather(xs, scores, rows)
    ref = (x.float() * scores.sum(-1, keepdim=True)).bfloat16()
    torch.testing.assert_close(out, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("R,E,N,K", [(1, 4, 128, 128), (700, 8, 256, 512), (4096, 8, 1024, 768), (50, 64, 128, 256)])
def test_grouped_gemm(R, E, N, K):
    torch.manual_seed(R)
    x = torch.randn(R, K, device="cuda").bfloat16()
    w = (torch.randn(E, N, K, device="cuda") / K**0.5).bfloat16()
    counts = torch.bincount(torch.randint(0, E, (R,), device="cuda"), minlength=E).int()
    if E > 2:
        counts[1] += counts[2]  # an empty expert in the middle
        counts[2] = 0
    y = moe_ops.hip_ops().grouped_gemm(x, w, counts)  # the in-tree MFMA kernel at every size
    ref = torch.empty(R, N, device="cuda")
    s = 0
    for e, c in enumerate(counts.tolist()):
        ref[s:s + c] = x[s:s + c].float() @ w[e].float().t()
        s += c
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    # size-dispatched entry (library grouped GEMM above GROUPED_LIBRARY_MIN_ROWS)
    torch.testing.assert_close(moe_ops.grouped_gemm(x, w, counts).float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("T,H,I,E,k", [(1, 256, 256, 8, 2), (200, 512, 384, 8, 2), (96, 256, 512, 16, 4)])
def test_moe_block_matches_reference(T, H, I, E, k):
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    torch.manual_seed(3)
    x = torch.randn(T, H, device="cuda").bfloat16()
    rw = (torch.randn(E, H, device="cuda") / H**0.5).bfloat16()
    w1 = (torch.randn(E, 2 * I, H, device="cuda") / H**0.5).bfloat16()
    w2 = (torch.randn(E, H, I, device="cuda") / I**0.5).bfloat16()
    act = lambda h: DF.gated_activation(h, "silu")  # noqa: E731
    assert moe_ops.native_moe_ok(x, rw, w1, w2, k)
    out = moe_ops.moe_block(x, rw, w1, w2, k, act, renormalize=True)
    f32act = lambda h: F.silu(h.float()[..., :I]) * h.float()[..., I:]  # noqa: E731
    scores, experts, _, _ = moe_ops.topk_gating(F.linear(x, rw), k, True)  # gating itself: test_topk_gating
    ref = moe_ops.moe_block_reference(x.float(), rw.float(), w1.float(), w2.float(), k, f32act, True,
                                      routing=(scores, experts))
    torch.testing.assert_close(out.float(), ref, rtol=3e-2, atol=3e-2)


def test_row_gathers():
    torch.manual_seed(4)
    table = torch.randn(1000, 256, device="cuda").bfloat16()
    pos_table = torch.randn(128, 256, device="cuda").bfloat16()
    ids = torch.randint(0, 1000, (77,), device="cuda")
    pos = torch.randint(0, 128, (77,), device="cuda")
    torch.testing.assert_close(moe_ops.embed_gather(table, ids), table[ids], rtol=0, atol=0)
    ref = (table[ids].float() + pos_table[pos].float()).bfloat16()
    torch.testing.assert_close(moe_ops.embed_gather(table, ids, pos_table, pos), ref, rtol=1e-2, atol=1e-2)
    idx = torch.randperm(1000, device="cuda")[:300]
    g = moe_ops.rows_gather(table, idx)
    assert torch.equal(g, table[idx])
    full = torch.zeros_like(table)
    moe_ops.rows_scatter(g, idx, full)
    assert torch.equal(full[idx], g)
    assert int((full.abs().sum(-1) > 0).sum()) == 300


def test_random_ltd_native_matches_index_ops():
    """Random-LTD token gather/scatter through the row kernels vs torch.gather/scatter, values and gradients."""
    from deepspeedsyclsupport_amd.runtime.data_pipeline.data_routing import basic_layer as BL
    torch.manual_seed(5)
    B, S, H, k = 3, 64, 128, 24
    lin = torch.nn.Linear(H, H).cuda().bfloat16()
    x = torch.randn(B, S, H, device="cuda").bfloat16().requires_grad_(True)
    idx = BL.token_sort_(torch.topk(torch.rand(B, S, device="cuda"), k, dim=-1).indices)
    flat = BL._flat(idx, S)
    part = BL._TokenGatherFn.apply(x, flat).view(B, k, H)
    out = BL._TokenScatterFn.apply(x, lin(part), flat)
    (out.float() ** 2).sum().backward()
    g_native = x.grad.clone()
    x.grad = None
    part_r = BL.token_gather(x, idx)
    out_r = BL.token_scatter_(x.clone(), lin(part_r), idx)
    (out_r.float() ** 2).sum().backward()
    assert torch.equal(out, out_r)
    torch.testing.assert_close(g_native, x.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("rows,S,k", [(16, 4096, 2048), (3, 100, 100), (8, 70000, 333), (2, 600000, 5000)])
def test_token_sort_kernel(rows, S, k):
    """Bitmap-compaction token sort (random-LTD token_sort_) == torch.sort on distinct positions, in place."""
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    keys = torch.rand(rows, S, device="cuda")
    idx = torch.topk(keys, k, dim=-1).indices.to(torch.int32).contiguous()
    ref = torch.sort(idx, dim=-1).values
    out = hip_ops().token_sort_(idx, S)
    assert out.data_ptr() == idx.data_ptr()
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
