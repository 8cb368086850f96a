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
        from deepspeedsyclsupport_amd.runtime.swap_tensor.optimizer_swapper import NvmeFlat
        sw = eng.optimizer.nvme_swapper
        assert sw is not None and sw.chunk == 5000 and sw.with_master
        # the fp32 master of the host partition is NVMe-resident, not a DRAM tensor
        assert all(isinstance(m, NvmeFlat) for m in eng.optimizer.master_host if m is not None)
        if offload[1] == 1.0:
            assert any(m is not None for m in eng.optimizer.master_host)
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
