"""Kernel objects of inference v2 (`inference/v2/kernels`): each against a plain fp32 PyTorch reference of the same
op — fp32 on the host (torch fallbacks of the same entry points), bf16 on the GPU (the HIP kernels)."""
import math

import pytest
import torch
import torch.nn.functional as F

from deepspeedsyclsupport_amd.inference.v2.inference_utils import ActivationType, DtypeEnum
from deepspeedsyclsupport_amd.inference.v2.kernels import (BlasLibLinear, BlockedFlashAttn, BlockedRotaryEmbeddings,
                                                           CUDABiasActivation, CUDAFPLN, CUDAFPPostLN, CUDAFPPreLN,
                                                           CUDAGatedActivation, CUDARMSNorm, CUDARMSPreNorm,
                                                           LinearBlockedKVCopy, MoEGather, MoEScatter,
                                                           RaggedEmbeddingKernel, RaggedLogitsGather,
                                                           RaggedTopKGating, AtomBuilder)
from deepspeedsyclsupport_amd.inference.v2.ragged import DSSequenceDescriptor, RaggedBatchWrapper

CASES = [pytest.param("cpu", torch.float32, id="cpu-fp32"),
         pytest.param("cuda", torch.bfloat16, id="gpu-bf16", marks=pytest.mark.gpu)]


def _tol(dtype):
    return dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)


def test_dtype_enum_spellings():
    assert DtypeEnum("bf16") is DtypeEnum.bf16 is DtypeEnum(torch.bfloat16) is DtypeEnum("torch.bfloat16")
    assert DtypeEnum("half").value == torch.float16
    with pytest.raises(ValueError):
        DtypeEnum("fp7")


@pytest.mark.parametrize("device,dtype", CASES)
def test_core_ops(device, dtype):
    torch.manual_seed(0)
    C, T = 256, 11
    x = torch.randn(T, C, device=device, dtype=dtype)
    y = torch.randn(T, C, device=device, dtype=dtype)
    g = (1 + 0.1 * torch.randn(C, device=device)).to(dtype)
    b = (0.1 * torch.randn(C, device=device)).to(dtype)
    tol = _tol(dtype)
    xf, yf, gf, bf = x.float(), y.float(), g.float(), b.float()

    out = torch.empty_like(x)
    CUDAFPLN(C, dtype)(out, x, g, b)
    torch.testing.assert_close(out.float(), F.layer_norm(xf, (C, ), gf, bf, 1e-5), **tol)
    CUDAFPPostLN(C, dtype)(out, x, y, g, b)
    torch.testing.assert_close(out.float(), F.layer_norm(xf + yf, (C, ), gf, bf, 1e-5), **tol)
    res = torch.empty_like(x)
    CUDAFPPreLN(C, dtype)(res, out, x, y, g, b)
    torch.testing.assert_close(res.float(), xf + yf, **tol)
    torch.testing.assert_close(out.float(), F.layer_norm(res.float(), (C, ), gf, bf, 1e-5), **tol)

    def rms(t):
        return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + 1e-5) * gf

    CUDARMSNorm(C, dtype)(out, x, g)
    torch.testing.assert_close(out.float(), rms(xf), **tol)
    CUDARMSPreNorm(C, dtype)(res, out, x, y, g)
    torch.testing.assert_close(res.float(), xf + yf, **tol)
    torch.testing.assert_close(out.float(), rms(res.float()), **tol)

    if dtype != torch.float32:
        act = x.clone()
        CUDABiasActivation(C, dtype, ActivationType.GELU)(act, b)
        torch.testing.assert_close(act.float(), F.gelu(xf + bf), **tol)
        act = x.clone()
        CUDABiasActivation(C, dtype, ActivationType.IDENTITY)(act, b)
        torch.testing.assert_close(act.float(), (x + b).float(), **tol)
    gu = torch.randn(T, 2 * C, device=device, dtype=dtype)
    go = torch.empty(T, C, device=device, dtype=dtype)
    CUDAGatedActivation(C, dtype, ActivationType.SiGLU)(go, gu)
    torch.testing.assert_close(go.float(), F.silu(gu.float()[:, :C]) * gu.float()[:, C:], **tol)

    w = torch.randn(96, C, device=device, dtype=dtype) * 0.05
    lo = torch.empty(T, 96, device=device, dtype=dtype)
    BlasLibLinear(dtype)(lo, x, w)
    torch.testing.assert_close(lo.float(), xf @ w.float().t(), **tol)

    with pytest.raises(ValueError):
        CUDAFPLN(C + 1, dtype)
    with pytest.raises(ValueError):
        CUDAGatedActivation(C, dtype, ActivationType.GELU)
    with pytest.raises(ValueError):
        CUDABiasActivation(C, torch.float32, ActivationType.GELU)


def _rope_ref(x, pos, rot, theta):
    """x [T, H, D] rotate-half over the first `rot` dims at positions pos [T]."""
    inv = 1.0 / (theta**(torch.arange(0, rot, 2, dtype=torch.float64) / rot))
    ang = torch.outer(pos.double(), inv)
    cos, sin = ang.cos().float()[:, None, :], ang.sin().float()[:, None, :]
    x = x.float()
    a, b, rest = x[..., :rot // 2], x[..., rot // 2:rot], x[..., rot:]
    return torch.cat([a * cos - b * sin, b * cos + a * sin, rest], -1)


@pytest.mark.parametrize("device,dtype", CASES)
@pytest.mark.parametrize("rotary", [True, False])
def test_ragged_attention_objects(device, dtype, rotary):
    """Two scheduling steps (two prompts; then one decode + one new prompt) through the KV-append and attention
    objects match dense causal attention over each sequence's full history."""
    torch.manual_seed(1)
    Hq, Hk, D, BS, theta = 4, 2, 64, 16, 10000.0
    kc = torch.zeros(32, Hk, BS, D, device=device, dtype=dtype)
    vc = torch.zeros_like(kc)
    rope = (BlockedRotaryEmbeddings(D, Hq, Hk, dtype, D, theta) if rotary else LinearBlockedKVCopy(D, Hq, Hk, dtype))
    attn = BlockedFlashAttn(D, dtype)
    batch = RaggedBatchWrapper(block_size=BS, device=torch.device(device))
    seqs = {u: DSSequenceDescriptor(u, BS) for u in (7, 8, 9)}
    history = {u: [] for u in seqs}      # per sequence: list of (q, k, v) fp32 [n, H, D] already rotated
    next_block = [0]

    def step(items):
        batch.clear()
        qkvs = []
        for u, n in items:
            s = seqs[u]
            need = s.blocks_needed(n)
            s.extend_kv_cache(range(next_block[0], next_block[0] + need))
            next_block[0] += need
            s.pre_forward(n)
            batch.insert_sequence(s, torch.zeros(n, dtype=torch.long))
            qkvs.append(torch.randn(n, (Hq + 2 * Hk) * D, device=device, dtype=dtype))
        batch.finalize()
        ordered = [qkvs[i] for i in batch.order]
        qkv = torch.cat(ordered)
        # reference: rotate at absolute positions, extend each sequence's history
        for j, i in enumerate(batch.order):
            u, n = items[i]
            q, k, v = ordered[j].float().view(n, Hq + 2 * Hk, D).split([Hq, Hk, Hk], 1)
            pos = torch.arange(seqs[u].seen_tokens, seqs[u].seen_tokens + n)
            if rotary:
                q, k = _rope_ref(q.cpu(), pos, D, theta), _rope_ref(k.cpu(), pos, D, theta)
            history[u].append((q.cpu(), k.cpu(), v.cpu()))
        q_rot = rope((kc, vc), qkv, batch)
        work, n_atoms = AtomBuilder()(None, batch)
        assert n_atoms == sum(-(-items[i][1] // 128) for i in batch.order[batch.meta.n_decode:])
        out = torch.empty(qkv.shape[0], Hq * D, device=device, dtype=dtype)
        attn(out, q_rot, (kc, vc), batch, 1.0 / math.sqrt(D))
        row = 0
        for i in batch.order:
            u, n = items[i]
            K = torch.cat([h[1] for h in history[u]]).repeat_interleave(Hq // Hk, 1)
            V = torch.cat([h[2] for h in history[u]]).repeat_interleave(Hq // Hk, 1)
            q = history[u][-1][0]
            L = K.shape[0]
            mask = torch.arange(L)[None, :] > (torch.arange(L - n, L)[:, None])
            sc = torch.einsum("nhd,lhd->hnl", q, K) / math.sqrt(D)
            sc = sc.masked_fill(mask[None], float("-inf"))
            ref = torch.einsum("hnl,lhd->nhd", sc.softmax(-1), V).reshape(n, Hq * D)
            torch.testing.assert_close(out[row:row + n].float().cpu(), ref,
                                       **(dict(rtol=3e-2, atol=3e-2) if dtype == torch.bfloat16 else
                                          dict(rtol=1e-4, atol=1e-4)))
            row += n
        for u, _ in items:
            seqs[u].post_forward()

    step([(7, 21), (8, 5)])
    step([(9, 140), (7, 1)])      # the decode of sequence 7 is moved in front of the new prompt
    assert batch.order == [1, 0] and batch.meta.n_decode == 1


@pytest.mark.parametrize("device,dtype", CASES)
def test_embedding_logits_and_moe_objects(device, dtype):
    torch.manual_seed(2)
    Hd, V, BS = 64, 50, 16
    table = torch.randn(V, Hd, device=device, dtype=dtype)
    ptable = torch.randn(40, Hd, device=device, dtype=dtype)
    batch = RaggedBatchWrapper(block_size=BS, device=torch.device(device))
    a, b = DSSequenceDescriptor(1, BS), DSSequenceDescriptor(2, BS)
    a.extend_kv_cache([0]), b.extend_kv_cache([1])
    a.seen_tokens = 3
    ta, tb = torch.randint(0, V, (4, )), torch.randint(0, V, (6, ))
    batch.insert_sequence(a, ta)
    batch.insert_sequence(b, tb)
    batch.finalize()
    emb = torch.empty(10, Hd, device=device, dtype=dtype)
    RaggedEmbeddingKernel(dtype, torch.int64, Hd)(emb, batch, table, ptable, position_embed_offset=2)
    ids = torch.cat([ta, tb]).to(device)
    pos = torch.cat([torch.arange(3, 7), torch.arange(0, 6)]).to(device) + 2
    torch.testing.assert_close(emb.float(), (table[ids].float() + ptable[pos].float()), **_tol(dtype))
    last = torch.empty(2, Hd, device=device, dtype=dtype)
    RaggedLogitsGather(Hd, dtype)(last, emb, batch)
    torch.testing.assert_close(last, emb[[3, 9]])
    assert batch.inflight_seq_descriptors(on_device=False).tolist() == [[0, 4, 3, 0], [4, 6, 0, 0]]
    assert batch.batch_metadata_buffer(on_device=False).tolist() == [10, 2]

    # MoE: gating -> scatter -> identity experts scaled by (expert id + 1) -> gather
    T, E, k = 10, 4, 2
    logits = torch.randn(T, E, device=device, dtype=dtype)
    counts = torch.empty(E, dtype=torch.int32, device=device)
    scores = torch.empty(T, k, dtype=torch.float32, device=device)
    assign = torch.empty(T, k, dtype=torch.int32, device=device)
    offs = torch.empty(T, k, dtype=torch.int32, device=device)
    RaggedTopKGating(dtype)(counts, scores, assign, offs, logits, batch)
    probs = logits.float().softmax(-1)
    rs, ra = probs.topk(k, -1)
    torch.testing.assert_close(scores, rs, rtol=1e-3, atol=1e-3)
    assert torch.equal(assign.long(), ra) and counts.sum().item() == T * k
    moe_in = torch.empty(T * k, Hd, device=device, dtype=dtype)
    cum = torch.empty(E, dtype=torch.int64, device=device)
    slots = torch.empty(T, k, dtype=torch.int32, device=device)
    MoEScatter(dtype, Hd)(moe_in, cum, slots, emb, counts, assign, offs)
    assert torch.equal(cum.cpu(), counts.cpu().long().cumsum(0))
    assert sorted(slots.reshape(-1).tolist()) == list(range(T * k))
    torch.testing.assert_close(moe_in[slots[:, 1].long()], emb)
    expert_of_row = torch.bucketize(torch.arange(T * k), cum.cpu(), right=True).to(device)
    moe_out = (moe_in.float() * (expert_of_row + 1)[:, None]).to(dtype)
    out = torch.empty(T, Hd, device=device, dtype=dtype)
    MoEGather(dtype, Hd)(out, moe_out, scores, slots, counts)
    ref = (emb.float()[:, None, :] * (ra + 1).float()[..., None] * rs[..., None]).sum(1)
    torch.testing.assert_close(out.float(), ref, **(dict(rtol=3e-2, atol=3e-2) if dtype == torch.bfloat16 else
                                                    dict(rtol=1e-5, atol=1e-5)))
