"""Universal checkpoint: streamed per-parameter conversion, tensor-parallel merge rules and their inverse, and a
world-4 -> world-2 reload that reproduces the native reload's next-step losses (reference
`checkpoint/ds_to_universal.py:87-286`, `universal_checkpoint.py:12-98`)."""
import os

import pytest
import torch

from deepspeedsyclsupport_amd.checkpoint import constants as CK
from deepspeedsyclsupport_amd.checkpoint.ds_to_universal import ds_to_universal, merge_tp_slices
from deepspeedsyclsupport_amd.checkpoint.universal_checkpoint import tp_slice

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama

INFO = {
    CK.TP_REPLICATED_PARAMETER_PATTERNS: [r".*norm\.weight"],
    CK.PARAMETER_TO_AVERAGE_PATTERNS: [r".*router\.bias"],
    CK.PARAMETER_WITH_ROW_PARALLELISM_PATTERNS: [r".*o_proj\.weight", r".*down_proj\.weight"],
    CK.VOCABULARY_PARAMETER_PATTERNS: [r".*embed_tokens\.weight"],
    CK.PARAMETER_WITH_2_SUB_PARAMS_CAT_DIM_0: [r".*gate_up_proj\.weight"],
    CK.ORIGINAL_VOCAB_SIZE: 50,
}


@pytest.mark.parametrize("tp_src,tp_dst", [(2, 1), (2, 4), (1, 2), (4, 2)])
def test_tp_merge_rules_and_their_inverse(tp_src, tp_dst):
    torch.manual_seed(0)
    H, I, V = 16, 32, 50
    vpad = lambda tp: -(-V // (8 * tp)) * 8 * tp  # noqa: E731  (vocab padded to a multiple of 8 per rank)
    full = {
        "layers.0.q_proj.weight": torch.randn(H, H),          # column parallel (dim 0)
        "layers.0.o_proj.weight": torch.randn(H, H),          # row parallel (dim 1)
        "layers.0.gate_up_proj.weight": torch.randn(2 * I, H),  # two fused sub-parameters
        "layers.0.norm.weight": torch.randn(H),               # replicated
        "layers.0.router.bias": torch.randn(8),               # averaged
        "embed_tokens.weight": torch.randn(V, H),             # vocabulary
    }

    def shard(name, t, tp, r):
        if "norm" in name or "router" in name:
            return t.clone()
        if "o_proj" in name:
            return t.chunk(tp, 1)[r].clone()
        if "gate_up" in name:
            return torch.cat([h.chunk(tp, 0)[r] for h in t.chunk(2, 0)], 0)
        if "embed" in name:
            return torch.nn.functional.pad(t, (0, 0, 0, vpad(tp) - V)).chunk(tp, 0)[r].clone()
        return t.chunk(tp, 0)[r].clone()

    used = set()
    for name, t in full.items():
        entry = merge_tp_slices(name, [shard(name, t, tp_src, r) for r in range(tp_src)], INFO, used)
        torch.testing.assert_close(entry[CK.PARAM], t, rtol=0, atol=0, msg=name)
        for r in range(tp_dst):
            want = shard(name, t, tp_dst, r)
            got = tp_slice(entry, want.shape, r, tp_dst)
            torch.testing.assert_close(got, want, rtol=0, atol=0, msg=f"{name} rank {r}")
    assert len(used) == 5  # every rule but the second row-parallel pattern (no such parameter here)
    with pytest.raises(ValueError):
        merge_tp_slices("layers.0.norm.weight", [torch.ones(4), torch.zeros(4)], INFO, set())


def _groups(model):
    decay = [p for n, p in model.named_parameters() if p.dim() >= 2]
    no_decay = [p for n, p in model.named_parameters() if p.dim() < 2]
    return [{"params": decay, "weight_decay": 0.1}, {"params": no_decay, "weight_decay": 0.0}]


def _save(stage, save):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    model = tiny_llama()
    eng, _, _, _ = ds.initialize(model=model, model_parameters=_groups(model),
                                 config=base_config(stage=stage, lr=1e-2, mb=2))
    for x in random_tokens(2, 2, 16, seed=5 + dist.get_rank()):
        eng.backward(eng(x, labels=x))
        eng.step()
    eng.save_checkpoint(save, tag="t")


def _resume(stage, save, tag, universal, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    cfg = base_config(stage=stage, lr=1e-2, mb=2)
    if universal:
        cfg["checkpoint"] = {"load_universal": True}
    model = tiny_llama(seed=11)
    eng, _, _, _ = ds.initialize(model=model, model_parameters=_groups(model), config=cfg)
    # a scatter that gathered would show up as per-parameter collectives: count them during the load
    calls = {"n": 0}
    orig = dist.all_gather_into_tensor

    def counting(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    dist.all_gather_into_tensor = counting
    try:
        eng.load_checkpoint(save, tag=tag)
    finally:
        dist.all_gather_into_tensor = orig
    n_params = sum(1 for _ in eng.module.parameters())
    # the module-state pass and the optimizer-state pass each refresh every persistent flat group once
    assert calls["n"] <= 2 * len(eng.optimizer.groups) < n_params, (calls["n"], len(eng.optimizer.groups), n_params)
    losses = []
    for x in random_tokens(2, 2, 16, seed=99):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    if dist.get_rank() == 0:
        torch.save(losses, out)


@pytest.mark.parametrize("stage_src,stage_dst", [(2, 3), (3, 1)])
def test_world4_to_universal_to_world2(stage_src, stage_dst, tmp_path):
    save = str(tmp_path / "ck")
    run_distributed(_save, 4, stage_src, save)
    stats = ds_to_universal(os.path.join(save, "t"), os.path.join(save, "t_universal"))
    assert stats["params"] == sum(1 for _ in tiny_llama().parameters())
    assert stats["peak_live_bytes"] <= 2 * stats["largest_param_bytes"]
    entry = torch.load(os.path.join(save, "t_universal", "zero", "model.norm.weight", "fp32.pt"), weights_only=True)
    assert set(entry) >= {CK.PARAM, CK.CAT_DIM}
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    run_distributed(_resume, 2, stage_dst, save, "t", False, a)
    run_distributed(_resume, 2, stage_dst, save, "t_universal", True, b)
    assert torch.load(b, weights_only=True) == pytest.approx(torch.load(a, weights_only=True), rel=1e-6)


def test_universal_from_reference_format_shards(tmp_path):
    """The converter reads the reference's own shard layout too (here: the files our exporter wrote)."""
    from deepspeedsyclsupport_amd.checkpoint import reference_format as rf
    save = str(tmp_path / "ck")
    run_distributed(_save, 2, 2, save)
    rf.export_checkpoint(save, "t")
    s1 = ds_to_universal(os.path.join(save, "t"), os.path.join(save, "u_native"))
    s2 = ds_to_universal(os.path.join(save, "reference_format", "t"), os.path.join(save, "u_ref"))
    assert s1["params"] == s2["params"]
    for name in os.listdir(os.path.join(save, "u_native", "zero")):
        d1, d2 = (os.path.join(save, u, "zero", name) for u in ("u_native", "u_ref"))
        if not os.path.isdir(d1):
            continue
        for key in ("fp32", "exp_avg", "exp_avg_sq"):
            x = torch.load(os.path.join(d1, f"{key}.pt"), weights_only=True)[CK.PARAM]
            y = torch.load(os.path.join(d2, f"{key}.pt"), weights_only=True)[CK.PARAM]
            torch.testing.assert_close(x, y, rtol=0, atol=0, msg=f"{name} {key}")
