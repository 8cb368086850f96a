"""ZeRO-Offload / Twin-Flow / ZeRO-Infinity optimizer offload (reference `tests/unit/runtime/zero/test_zero.py`
offload cases, `test_zeropp`/`test_nvme_checkpointing`): host-stepped partitions (native CPU Adam, optionally with
moments streamed from NVMe files) must reproduce the all-device run, and checkpoints must round-trip."""
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
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    if offload and offload[0] == "nvme":
        assert eng.optimizer.nvme_swapper is not None
        eng.optimizer.nvme_swapper.chunk = 5000  # force several chunks through the read-ahead pipeline
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
