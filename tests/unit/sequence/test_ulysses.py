"""Ulysses SP (no test exists in the reference: SURVEY §4 gap). SP=2 over gloo vs single-process full-sequence."""
import pytest
import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama

STEPS, B, S = 3, 2, 32


def _ref():
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    model = tiny_llama(num_attention_heads=4, num_key_value_heads=2)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    data = random_tokens(STEPS, B, S, seed=7)
    losses = []
    for x in data:
        opt.zero_grad()
        labels = torch.full_like(x, -100)
        labels[:, :-1] = x[:, 1:]
        h = model.model(x)
        logits = model.lm_head(h)
        per = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), labels.reshape(-1),
                                                ignore_index=-100, reduction="none").view(B, S)
        valid = (labels != -100).float()
        half = S // 2
        l0 = (per[:, :half] * valid[:, :half]).sum() / valid[:, :half].sum()
        l1 = (per[:, half:] * valid[:, half:]).sum() / valid[:, half:].sum()
        loss = (l0 + l1) / 2
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        losses.append(float(loss))
    return losses


def _sp_run(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.parallel import groups
    from deepspeedsyclsupport_amd.sequence.layer import enable_sequence_parallel, shard_sequence
    model = tiny_llama(num_attention_heads=4, num_key_value_heads=2)
    cfg = base_config(stage=2, lr=1e-2, mb=B)
    cfg["sequence_parallel"] = {"size": 2}
    cfg["train_batch_size"] = B  # dp = world / sp = 1
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    assert enable_sequence_parallel(eng.module, groups._get_sequence_parallel_group()) == 2
    losses = []
    for x in random_tokens(STEPS, B, S, seed=7):
        inp, lab, off = shard_sequence(x, x, groups._get_sequence_parallel_group())
        loss = eng(inp, labels=lab, pos_offset=off, shift_labels=False)
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / 2)
    if dist.get_rank() == 0:
        torch.save(losses, out)


def test_ulysses_matches_full_sequence(tmp_path):
    out = str(tmp_path / "l.pt")
    run_distributed(_sp_run, 2, out)
    got = torch.load(out)
    ref = _ref()
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-5), (got, ref)


def _a2a_roundtrip():
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.sequence.layer import _FusedQKVToSeq, _SeqToHeads, single_all_to_all
    torch.manual_seed(dist.get_rank())
    q = torch.randn(2, 4, 8, 16, requires_grad=True)
    k = torch.randn(2, 2, 8, 16, requires_grad=True)
    v = torch.randn(2, 2, 8, 16, requires_grad=True)
    qs, ks, vs = _FusedQKVToSeq.apply(None, q, k, v)
    assert qs.shape == (2, 2, 16, 16) and ks.shape == (2, 1, 16, 16)
    back = _SeqToHeads.apply(None, qs)
    torch.testing.assert_close(back, q)
    (qs.sum() * 2 + ks.sum() * 3 + vs.sum() * 4).backward()
    assert torch.all(q.grad == 2) and torch.all(k.grad == 3) and torch.all(v.grad == 4)
    x = torch.randn(8, 2, 4, 16)  # [s, b, h, d]
    y = single_all_to_all(x, 2, 0, None)
    assert y.shape == (16, 2, 2, 16)
    z = single_all_to_all(y, 0, 2, None)
    torch.testing.assert_close(z, x)


def test_fused_qkv_all_to_all_roundtrip():
    run_distributed(_a2a_roundtrip, 2)
