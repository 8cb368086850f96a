"""ZeRO-3 with parameters the optimizer does not own (reference `tests/unit/runtime/zero/test_zero.py`
TestZeroFrozenWeights, `tests/unit/checkpoint/test_zero_optimizer.py` frozen-weight cases): a frozen base model with
trained adapters is the common fine-tuning setup, and the frozen weights are most of the memory. They are partitioned,
fetched around their module's forward / backward and released again, homed on the host with offload_param, saved as
per-rank shards and restored under another data-parallel size — and never change."""
import os

import pytest
import torch
import torch.nn as nn

from ..common import run_distributed

H = 32


class Block(nn.Module):
    """Frozen base projection + trained low-rank adapter; one mixed module (frozen weight, trained bias) too."""

    def __init__(self):
        super().__init__()
        self.base = nn.Linear(H, H)
        self.down = nn.Linear(H, 4, bias=False)
        self.up = nn.Linear(4, H, bias=False)
        self.mixed = nn.Linear(H, H)

    def forward(self, x):
        x = torch.tanh(self.base(x) + self.up(self.down(x)))
        return torch.tanh(self.mixed(x))


def build(seed=0):
    torch.manual_seed(seed)
    m = nn.Sequential(nn.Linear(16, H), Block(), Block(), nn.Linear(H, 4))
    return m


def freeze(m):
    for p in m[0].parameters():          # first layer frozen: no input of it needs a gradient
        p.requires_grad_(False)
    for blk in (m[1], m[2]):
        for p in blk.base.parameters():
            p.requires_grad_(False)
        blk.mixed.weight.requires_grad_(False)
    return m


def data(n, rank=0, seed=5):
    g = torch.Generator().manual_seed(seed + rank)
    return [(torch.randn(4, 16, generator=g), torch.randint(0, 4, (4, ), generator=g)) for _ in range(n)]


def cfg(stage=3, **zero):
    z = {"stage": stage, "stage3_param_persistence_threshold": 0}
    z.update(zero)
    return {"train_micro_batch_size_per_gpu": 4, "steps_per_print": 1000, "zero_optimization": z,
            "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.0}}}


def _reference(world, steps):
    """Plain PyTorch: the same model, the global batch = every rank's batch."""
    m = freeze(build())
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-2, weight_decay=0.0)
    per_rank = [data(steps, r) for r in range(world)]
    losses = []
    for s in range(steps):
        opt.zero_grad()
        tot = 0.0
        for r in range(world):
            x, y = per_rank[r][s]
            loss = nn.functional.cross_entropy(m(x), y) / world
            loss.backward()
            tot += float(loss)
        opt.step()
        losses.append(tot)
    return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}


def _train(out, use_init, zero_extra, steps=3):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    c = cfg(**zero_extra)
    if use_init:
        with ds.zero.Init(config_dict_or_path=c):
            m = build()
    else:
        m = build()
    freeze(m)
    eng, *_ = ds.initialize(model=m, config=c, model_parameters=[p for p in m.parameters() if p.requires_grad])
    opt = eng.optimizer
    frozen = [p for p in m.parameters() if not p.requires_grad]
    assert len(opt.frozen_groups) == 5 and sum(len(g.params) for g in opt.frozen_groups) == len(frozen)
    losses = []
    for x, y in data(steps, dist.get_rank()):
        loss = nn.functional.cross_entropy(eng(x), y)
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / dist.get_world_size())
    # released again: neither trained nor frozen weights stay gathered between steps
    assert all(p.numel() == 0 for p in m.parameters())
    assert all(g.full is None for g in opt.all_groups if not g.persistent)
    if zero_extra.get("offload_param"):
        assert all(g.shard.device.type == "cpu" for g in opt.frozen_groups)
    w = {n: safe_get_full_fp32_param(p).cpu() for n, p in m.named_parameters()}
    with ds.zero.GatheredParameters(frozen):
        assert all(p.numel() > 0 for p in frozen)
    full = eng.consolidated_16bit_state_dict()  # the 16-bit export gathers trained and frozen groups alike
    if dist.get_rank() == 0:
        assert set(full) == set(w) and all(torch.equal(full[n].float(), w[n]) for n in w)
        torch.save({"losses": losses, "w": w}, out)


@pytest.mark.parametrize("world,use_init,zero_extra", [
    (2, False, {}),
    (2, True, {}),
    (2, False, {"offload_param": {"device": "cpu"}}),
    (1, True, {"offload_param": {"device": "cpu"}}),
])
def test_frozen_parameters_are_partitioned_and_training_matches(world, use_init, zero_extra, tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_train, world, out, use_init, zero_extra)
    got = torch.load(out)
    losses, ref = _reference(world, 3)
    assert got["losses"] == pytest.approx(losses, rel=1e-5, abs=1e-6)
    init = freeze(build()).state_dict()
    for n, v in ref.items():
        torch.testing.assert_close(got["w"][n], v, rtol=1e-5, atol=1e-6, msg=n)
    for n in ("0.weight", "1.base.weight", "2.mixed.weight"):
        assert torch.equal(got["w"][n], init[n]), n  # frozen means frozen


def _save(save_dir, out, exclude):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    m = freeze(build())
    with torch.no_grad():  # make the frozen weights differ from a fresh build, so a load has something to prove
        for p in m.parameters():
            if not p.requires_grad:
                p.add_(0.5)
    eng, *_ = ds.initialize(model=m, config=cfg(), model_parameters=[p for p in m.parameters() if p.requires_grad])
    for x, y in data(2, dist.get_rank()):
        eng.backward(nn.functional.cross_entropy(eng(x), y))
        eng.step()
    eng.save_checkpoint(save_dir, tag="t", exclude_frozen_parameters=exclude)
    w = {n: safe_get_full_fp32_param(p).cpu() for n, p in m.named_parameters()}
    nxt = []
    for x, y in data(4, dist.get_rank())[2:]:
        loss = nn.functional.cross_entropy(eng(x), y)
        eng.backward(loss)
        eng.step()
        nxt.append(float(loss.detach()))
    if dist.get_rank() == 0:
        torch.save({"w": w, "next": nxt}, out)


def _load(save_dir, out, strict):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    m = freeze(build())
    eng, *_ = ds.initialize(model=m, config=cfg(), model_parameters=[p for p in m.parameters() if p.requires_grad])
    eng.load_checkpoint(save_dir, load_module_strict=strict)
    w = {n: safe_get_full_fp32_param(p).cpu() for n, p in m.named_parameters()}
    nxt = []
    for x, y in data(4, dist.get_rank())[2:]:
        loss = nn.functional.cross_entropy(eng(x), y)
        eng.backward(loss)
        eng.step()
        nxt.append(float(loss.detach()))
    if dist.get_rank() == 0:
        torch.save({"w": w, "next": nxt}, out)


@pytest.mark.parametrize("load_world", [2, 1])
def test_frozen_shards_checkpoint_roundtrip(load_world, tmp_path):
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    ck = str(tmp_path / "ck")
    run_distributed(_save, 2, ck, a, False)
    run_distributed(_load, load_world, ck, b, True)
    saved, loaded = torch.load(a), torch.load(b)
    for n in saved["w"]:
        assert torch.equal(saved["w"][n], loaded["w"][n]), n
    if load_world == 2:
        assert loaded["next"] == pytest.approx(saved["next"], rel=1e-6)
    # the offline consolidation tool sees trained AND frozen parameters
    from deepspeedsyclsupport_amd.utils.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
    full = get_fp32_state_dict_from_zero_checkpoint(ck, "t")
    for n in saved["w"]:
        torch.testing.assert_close(full[n], saved["w"][n], rtol=0, atol=0, msg=n)
    only_trained = get_fp32_state_dict_from_zero_checkpoint(ck, "t", exclude_frozen_parameters=True)
    assert "1.base.weight" not in only_trained and "1.down.weight" in only_trained


def test_exclude_frozen_parameters_on_save(tmp_path):
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    ck = str(tmp_path / "ck")
    run_distributed(_save, 2, ck, a, True)
    sd = torch.load(os.path.join(ck, "t", "zero_pp_rank_0_mp_rank_00_optim_states.pt"),
                    weights_only=False)["optimizer_state_dict"]
    assert "frozen_shards" not in sd
    run_distributed(_load, 2, ck, b, False)
    saved, loaded = torch.load(a), torch.load(b)
    init = freeze(build()).state_dict()
    for n in saved["w"]:
        if n in ("0.weight", "0.bias", "1.base.weight", "1.base.bias", "1.mixed.weight", "2.base.weight",
                 "2.base.bias", "2.mixed.weight"):
            assert torch.equal(loaded["w"][n], init[n]), n      # not in the checkpoint: the model's own values stay
        else:
            assert torch.equal(loaded["w"][n], saved["w"][n]), n


def _qnt(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.zero import zeropp
    calls = {"n": 0, "frozen_only": True}
    orig = zeropp.quantized_all_gather

    def spy(full, shard, group):
        calls["n"] += 1
        return orig(full, shard, group)

    zeropp.quantized_all_gather = spy
    m = freeze(build())
    eng, *_ = ds.initialize(model=m, config=cfg(zero_quantized_nontrainable_weights=True),
                            model_parameters=[p for p in m.parameters() if p.requires_grad])
    losses = []
    for x, y in data(3, dist.get_rank()):
        loss = nn.functional.cross_entropy(eng(x), y)
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / dist.get_world_size())
    n_frozen_fetches = sum(1 for g in eng.optimizer.frozen_groups)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "calls": calls["n"], "frozen_groups": n_frozen_fetches}, out)


def test_quantized_nontrainable_weights_gather(tmp_path):
    """`zero_quantized_nontrainable_weights`: only the frozen groups travel as int8 blocks; training follows the
    16-bit run within quantisation noise."""
    out = str(tmp_path / "r.pt")
    run_distributed(_qnt, 2, out)
    r = torch.load(out)
    ref, _ = _reference(2, 3)
    assert r["calls"] >= r["frozen_groups"] * 3          # every step fetches every frozen group at least once
    assert r["calls"] <= r["frozen_groups"] * 3 * 2      # ... and only those (forward + backward fetches)
    assert r["losses"] == pytest.approx(ref, rel=0.05, abs=0.05)
    assert r["losses"] != pytest.approx(ref, rel=1e-7, abs=1e-9)
