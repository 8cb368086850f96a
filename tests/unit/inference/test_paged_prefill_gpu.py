"""Ragged paged flash-prefill kernel (csrc/attn/paged_prefill.hip) vs an fp32 reference over the same paged cache:
mixed chunk lengths and cached prefixes, GQA, ALiBi, sliding windows, cache block sizes 16 / 64."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(lens, starts, Hq, Hk, BS, alibi, window, seed=0, D=128):
    from deepspeedsyclsupport_amd.inference.model_implementations.transformer import RaggedMeta, alibi_slopes
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    g = torch.Generator(device="cuda").manual_seed(seed)
    S = len(lens)
    need = [-(-(st + n) // BS) for st, n in zip(starts, lens)]
    nblocks = sum(need) + 3
    kc = torch.randn(nblocks, Hk, BS, D, device="cuda", generator=g).bfloat16()
    vc = torch.randn(nblocks, Hk, BS, D, device="cuda", generator=g).bfloat16()
    perm = torch.randperm(nblocks, generator=torch.Generator().manual_seed(seed)).tolist()
    blocks, o = [], 0
    for nb in need:
        blocks.append(perm[o:o + nb])
        o += nb
    meta = RaggedMeta.build(starts, lens, blocks, 0, BS, torch.device("cuda"))
    T = sum(lens)
    q = torch.randn(T, Hq, D, device="cuda", generator=g).bfloat16()
    slopes = alibi_slopes(Hq).cuda() if alibi else None
    scale = 1.0 / math.sqrt(D)
    out = hip_ops().paged_prefill(q, kc, vc, meta.block_tables, meta.start_pos, meta.cu_q, meta.work, slopes, window,
                                  scale)
    torch.cuda.synchronize()
    for i in range(S):
        a, b = meta.cu_host[i], meta.cu_host[i + 1]
        L = starts[i] + lens[i]
        ids = torch.tensor(blocks[i], device="cuda")
        k = kc[ids].transpose(0, 1).reshape(Hk, -1, D)[:, :L].float()
        v = vc[ids].transpose(0, 1).reshape(Hk, -1, D)[:, :L].float()
        k, v = k.repeat_interleave(Hq // Hk, 0), v.repeat_interleave(Hq // Hk, 0)
        qi = q[a:b].float().transpose(0, 1)  # [Hq, n, D]
        s = qi @ k.transpose(1, 2) * scale
        qpos = torch.arange(starts[i], L, device="cuda")
        kpos = torch.arange(L, device="cuda")
        if alibi:
            s = s + slopes[:, None, None] * (kpos[None, None, :] - qpos[None, :, None]).float()
        bad = kpos[None, :] > qpos[:, None]
        if window:
            bad = bad | (kpos[None, :] <= qpos[:, None] - window)
        s = s.masked_fill(bad[None], float("-inf"))
        ref = torch.softmax(s, -1) @ v
        torch.testing.assert_close(out[a:b].float().transpose(0, 1), ref, rtol=2e-2, atol=2e-2,
                                   msg=lambda m: f"seq {i} (start {starts[i]}, n {lens[i]}): {m}")


@pytest.mark.parametrize("Hq,Hk", [(8, 8), (8, 2)])
@pytest.mark.parametrize("BS", [16, 64])
def test_paged_prefill_mixed_chunks(Hq, Hk, BS):
    _case([37, 1, 200, 129, 64], [0, 100, 0, 70, 333], Hq, Hk, BS, alibi=False, window=0)


@pytest.mark.parametrize("window", [0, 37, 200])
def test_paged_prefill_alibi_window(window):
    _case([90, 300, 5], [0, 20, 400], 4, 4, 64, alibi=True, window=window, seed=window)


def test_paged_prefill_long_prefix():
    _case([256, 17], [3000, 4095], 8, 1, 64, alibi=False, window=0, seed=3)


@pytest.mark.parametrize("D", [64, 80, 96, 256])
@pytest.mark.parametrize("alibi,window", [(False, 0), (True, 70)])
def test_paged_prefill_head_dims(D, alibi, window):
    """GPT-2 / Phi / GPT-NeoX-20B / GPT-J head sizes through the same kernel template."""
    _case([37, 1, 200, 129, 64], [0, 100, 0, 70, 333], 8, 2, 64, alibi=alibi, window=window, seed=D, D=D)


def test_uniform_tables_are_cached():
    from deepspeedsyclsupport_amd.inference.model_implementations import transformer as tr
    a = tr._uniform_tables(3, 300, torch.device("cuda"))
    b = tr._uniform_tables(3, 300, torch.device("cuda"))
    assert a[0] is b[0] and a[1] is b[1]
    assert a[0].tolist() == [0, 300, 600, 900]
    assert a[1].tolist() == [[s, q] for s in range(3) for q in range(3)]
