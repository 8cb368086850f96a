"""ZeRO-Offload / Twin-Flow / ZeRO-Infinity optimizer offload (reference `tests/unit/runtime/zero/test_zero.py`
offload cases, `test_zeropp`/`test_nvme_checkpointing`): host-stepped partitions (native CPU Adam, optionally with
the fp32 master and moments streamed from NVMe files) must reproduce the all-device run, and checkpoints must
round-trip."""
import pytest
import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama


def _run(offload, out, nvme_dir, ckpt_dir):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    cfg = base_config(stage=3, lr=1e-2, mb=2, clip=1.0)
    if offload is not None:
        device, ratio = offload
        cfg["zero_optimization"]["offload_optimizer"] = {"device": device, "ratio": ratio, "nvme_path": nvme_dir}
        if device == "nvme":
            cfg["zero_optimization"]["sub_group_size"] = 5000  # several chunks through the read-ahead pipeline
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    if offload and offload[0] == "nvme":
        sw, off = eng.optimizer.nvme_swapper, eng.optimizer.off
        assert sw is not None and sw.chunk == 6144 and sw.with_master  # 5000 rounded up to the I/O alignment
        # the fp32 master and moments of the offloaded partition are NVMe-resident, not DRAM tensors
        assert off is not None and all(r == 0 for r in off.res) and sw.bytes_on_disk() > 0
        if offload[1] == 1.0:
            assert sum(off.n) == sum(r[1] - r[0] for g in eng.optimizer.groups for r in g.runs)
    losses = []
    for x in random_tokens(3, 2, 16, seed=40 + dist.get_rank()):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    w = {n: safe_get_full_fp32_param(p) for n, p in eng.module.named_parameters()}
    m = {n: safe_get_full_optimizer_state(p, "exp_avg") for n, p in eng.module.named_parameters()}
    if ckpt_dir:
        eng.save_checkpoint(ckpt_dir, tag="t")
        eng2, _, _, _ = ds.initialize(model=tiny_llama(seed=5), config=cfg)
        eng2.load_checkpoint(ckpt_dir, tag="t")
        for n, p in eng2.module.named_parameters():
            torch.testing.assert_close(safe_get_full_fp32_param(p), w[n], rtol=0, atol=0)
            torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg"), m[n], rtol=0, atol=0)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "w": w}, out)


@pytest.mark.parametrize("offload", [("cpu", 1.0), ("cpu", 0.5), ("nvme", 1.0), ("nvme", 0.5)])
def test_optimizer_offload_matches_device(offload, tmp_path):
    ref_out, got_out = str(tmp_path / "ref.pt"), str(tmp_path / "got.pt")
    run_distributed(_run, 2, None, ref_out, None, None)
    run_distributed(_run, 2, offload, got_out, str(tmp_path / "nvme"), str(tmp_path / "ckpt"))
    ref, got = torch.load(ref_out, weights_only=True), torch.load(got_out, weights_only=True)
    assert got["losses"] == pytest.approx(ref["losses"], rel=1e-5, abs=1e-6)
    for n in ref["w"]:
        torch.testing.assert_close(got["w"][n], ref["w"][n], rtol=1e-5, atol=1e-6, msg=n)


def _run_param_offload(pdev, opt_dev, out, nvme_dir, ckpt_dir):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    cfg = base_config(stage=3, lr=1e-2, mb=2, clip=1.0)
    cfg["zero_optimization"]["stage3_param_persistence_threshold"] = 100
    if pdev is not None:
        cfg["zero_optimization"]["offload_param"] = {"device": pdev, "nvme_path": nvme_dir}
    if opt_dev is not None:
        cfg["zero_optimization"]["offload_optimizer"] = {"device": opt_dev, "nvme_path": nvme_dir}
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    opt = eng.optimizer
    if pdev is not None:
        assert opt.offload_param and opt.coordinator is not None
        off = [g for g in opt.groups if not g.persistent]
        assert off, "expected offloaded (non-persistent) groups"
        if pdev == "nvme":
            assert opt.param_store is not None and opt.param_store.bytes_on_disk() > 0
    losses = []
    for x in random_tokens(3, 2, 16, seed=40 + dist.get_rank()):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    if pdev is not None:  # after the step everything but the persistent group is released again
        assert all(g.full is None for g in opt.groups if not g.persistent)
    w = {n: safe_get_full_fp32_param(p) for n, p in eng.module.named_parameters()}
    if ckpt_dir:
        eng.save_checkpoint(ckpt_dir, tag="t")
        eng2, _, _, _ = ds.initialize(model=tiny_llama(seed=5), config=cfg)
        eng2.load_checkpoint(ckpt_dir, tag="t")
        for n, p in eng2.module.named_parameters():
            torch.testing.assert_close(safe_get_full_fp32_param(p), w[n], rtol=0, atol=0)
        x = random_tokens(1, 2, 16, seed=99)[0]
        torch.testing.assert_close(eng2(x, labels=x), eng(x, labels=x), rtol=0, atol=0)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "w": w}, out)


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("pdev,opt_dev", [("cpu", None), ("cpu", "cpu"), ("nvme", None), ("nvme", "nvme")])
def test_param_offload_matches_device(world, pdev, opt_dev, tmp_path):
    """ZeRO-Infinity offload_param (reference `partitioned_param_swapper.py`): shards homed on the host / NVMe and
    streamed in per module must train exactly like the device-resident ZeRO-3 run."""
    ref_out, got_out = str(tmp_path / "ref.pt"), str(tmp_path / "got.pt")
    run_distributed(_run_param_offload, world, None, None, ref_out, None, None)
    run_distributed(_run_param_offload, world, pdev, opt_dev, got_out, str(tmp_path / "nvme"), str(tmp_path / "ck"))
    ref, got = torch.load(ref_out, weights_only=True), torch.load(got_out, weights_only=True)
    assert got["losses"] == pytest.approx(ref["losses"], rel=1e-5, abs=1e-6)
    for n in ref["w"]:
        torch.testing.assert_close(got["w"][n], ref["w"][n], rtol=1e-5, atol=1e-6, msg=n)


# ------------------------------------------------------------------------------------------------ tiers / split
def _run_tiers(variant, out, nvme_dir, ckpt_dir):
    """variant: dict(stage, gas, dtype, offload=None | dict(offload_optimizer keys), split=bool, steps)."""
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    gas = variant.get("gas", 1)
    cfg = base_config(stage=variant.get("stage", 3), lr=1e-2, mb=2, gas=gas, clip=1.0,
                      dtype=variant.get("dtype", "fp32"))
    cfg["zero_optimization"]["sub_group_size"] = 4096
    if variant.get("offload"):
        oc = dict(variant["offload"])
        oc.setdefault("nvme_path", nvme_dir)
        cfg["zero_optimization"]["offload_optimizer"] = oc
    if variant.get("split"):
        cfg["bf16"]["split_master_weights"] = True
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    opt = eng.optimizer
    if variant.get("offload") and variant["offload"].get("max_in_cpu"):
        off = opt.off
        assert sum(off.res) == min(variant["offload"]["max_in_cpu"], sum(off.n)) and sum(off.n) > sum(off.res) > 0
    losses = []
    data = random_tokens(variant.get("steps", 3) * gas, 2, 16, seed=40 + dist.get_rank())
    for x in data:
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    w = {n: safe_get_full_fp32_param(p) for n, p in eng.module.named_parameters()}
    m = {n: safe_get_full_optimizer_state(p, "exp_avg_sq") for n, p in eng.module.named_parameters()}
    if variant.get("split"):
        # the 16-bit weight is the fp32 master rounded to nearest (ties away from zero): |w16 - master| <= ulp/2
        sd = eng.consolidated_16bit_state_dict(rank0_only=False)
        for n, v in w.items():
            w16 = sd[n].float().to(v.device)
            ulp = torch.maximum(v.abs(), torch.full_like(v, 1e-30)) * 2.0**-8
            assert bool(((w16 - v).abs() <= ulp).all()), n
    if ckpt_dir:
        eng.save_checkpoint(ckpt_dir, tag="t")
        eng2, _, _, _ = ds.initialize(model=tiny_llama(seed=5), config=cfg)
        eng2.load_checkpoint(ckpt_dir, tag="t")
        for n, p in eng2.module.named_parameters():
            torch.testing.assert_close(safe_get_full_fp32_param(p), w[n], rtol=0, atol=0)
            torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg_sq"), m[n], rtol=0, atol=0)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "w": w}, out)


def _compare_tiers(tmp_path, world, ref_variant, variant, rtol=1e-5, atol=1e-6, mean_only=False):
    ref_out, got_out = str(tmp_path / "ref.pt"), str(tmp_path / "got.pt")
    run_distributed(_run_tiers, world, ref_variant, ref_out, None, None)
    run_distributed(_run_tiers, world, variant, got_out, str(tmp_path / "nvme"), str(tmp_path / "ckpt"))
    ref, got = torch.load(ref_out, weights_only=True), torch.load(got_out, weights_only=True)
    assert got["losses"] == pytest.approx(ref["losses"], rel=max(rtol, 1e-5), abs=1e-6)
    for n in ref["w"]:
        if mean_only:  # 16-bit runs: Adam turns a rounding-level gradient difference into a full lr-sized step
            assert float((got["w"][n] - ref["w"][n]).abs().mean()) < atol, n
        else:
            torch.testing.assert_close(got["w"][n], ref["w"][n], rtol=rtol, atol=atol, msg=n)


@pytest.mark.parametrize("world", [1, 2])
def test_three_tier_offload_matches_device(world, tmp_path):
    """device + host DRAM (max_in_cpu) + NVMe tail in one optimizer: same training as the all-device run."""
    _compare_tiers(tmp_path, world, dict(stage=3),
                   dict(stage=3, offload={"device": "nvme", "ratio": 0.7, "max_in_cpu": 20000}))


@pytest.mark.parametrize("stage", [2, 3])
def test_offload_with_gradient_accumulation(stage, tmp_path):
    """gas > 1 under partitioned ZeRO-2/3: micro-step gradients are summed in the fp32 host accumulator."""
    _compare_tiers(tmp_path, 2, dict(stage=stage, gas=2), dict(stage=stage, gas=2, offload={"device": "cpu",
                                                                                            "ratio": 0.6}))


@pytest.mark.parametrize("offload", [None, {"device": "cpu", "ratio": 0.5},
                                     {"device": "nvme", "ratio": 1.0, "max_in_cpu": 30000}])
def test_split_master_weights(offload, tmp_path):
    """bf16 weight + int16 residual masters train like fp32 masters (identical arithmetic; the weights differ from
    the fp32-master run only where rounding hits an exact tie) on every tier, and round-trip through checkpoints."""
    _compare_tiers(tmp_path, 2, dict(stage=3, dtype="bf16"),
                   dict(stage=3, dtype="bf16", split=True, offload=offload), rtol=2e-2, atol=2e-3, mean_only=True)


def test_split_master_cpu_adam_is_exact():
    """cpu_adam_update_split reproduces cpu_adam_update bit for bit: join(hi, lo) == fp32 master after every step."""
    from deepspeedsyclsupport_amd.ops.native import cpu_ops
    from deepspeedsyclsupport_amd.runtime.zero.offload import split_cut, split_join
    torch.manual_seed(0)
    n = 70001
    p = torch.randn(n) * 0.05
    hi, lo = split_cut(p)
    assert torch.equal(split_join(hi, lo), p)
    m, v = torch.zeros(n), torch.zeros(n)
    m2, v2 = torch.zeros(n), torch.zeros(n)
    for step in range(1, 5):
        g = (torch.randn(n) * 1e-2).bfloat16()
        lp = torch.empty(n, dtype=torch.bfloat16)
        cpu_ops().cpu_adam_update(p, m, v, g, lp, step, 1e-2, 0.9, 0.95, 1e-8, 0.1, True, True, 0.5)
        stage = g.clone()  # gradient in, weight out through the same buffer
        cpu_ops().cpu_adam_update_split(lo, m2, v2, stage, hi, stage, step, 1e-2, 0.9, 0.95, 1e-8, 0.1, True, True,
                                        0.5)
        hi = stage.clone()
        assert torch.equal(split_join(hi, lo), p) and torch.equal(m, m2) and torch.equal(v, v2)
        assert bool(((hi.float() - p).abs() <= p.abs() * 2.0**-8).all())
