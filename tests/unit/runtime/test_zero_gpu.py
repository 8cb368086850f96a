"""ZeRO engine on the GPU against plain PyTorch (the device path: fused HIP Adam, HIP norm/act/RoPE/CE kernels,
flat buffers, comm streams). fp32 must track torch.optim.AdamW tightly; bf16 must follow the fp32 trajectory."""
import pytest
import torch

from ..simple_model import tiny_llama

pytestmark = pytest.mark.gpu


def _data(n, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, 128, (2, 32), generator=g).cuda() for _ in range(n)]


def _torch_ref(steps, lr):
    torch.manual_seed(0)
    m = tiny_llama(hidden_size=128, intermediate_size=256, num_attention_heads=4).cuda()
    opt = torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=0.01)
    out = []
    for x in _data(steps, 5):
        loss = m(x, labels=x)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        out.append(float(loss))
    return out


def _engine(stage, dtype, steps, lr, zero_extra=None):
    import deepspeedsyclsupport_amd as ds
    from ..simple_model import base_config
    torch.manual_seed(0)
    m = tiny_llama(hidden_size=128, intermediate_size=256, num_attention_heads=4)
    cfg = base_config(stage=stage, lr=lr, mb=2, clip=1.0, dtype=dtype)
    cfg["zero_optimization"].update(zero_extra or {})
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    out = []
    for x in _data(steps, 5):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        out.append(float(loss))
    return out


@pytest.mark.parametrize("stage", [0, 2, 3])
def test_engine_fp32_matches_torch(stage):
    ref = _torch_ref(6, 3e-3)
    got = _engine(stage, "fp32", 6, 3e-3)
    assert got == pytest.approx(ref, rel=2e-3, abs=2e-3), (got, ref)


def test_engine_bf16_tracks_fp32():
    ref = _torch_ref(6, 3e-3)
    got = _engine(3, "bf16", 6, 3e-3)
    assert got == pytest.approx(ref, rel=3e-2, abs=3e-2), (got, ref)


@pytest.mark.parametrize("opt_dev", [None, "cpu"])
@pytest.mark.parametrize("pdev", ["cpu", "nvme"])
def test_param_offload_gpu_matches_device(pdev, opt_dev, tmp_path):
    """ZeRO-Infinity on the device path: pinned-host / NVMe-mapped shards streamed H2D on the all-gather stream,
    device Adam writing back through a device temp (or native CPU Adam for the offloaded optimizer)."""
    extra = {"stage3_param_persistence_threshold": 1000,
             "offload_param": {"device": pdev, "nvme_path": str(tmp_path)}}
    if opt_dev:
        extra["offload_optimizer"] = {"device": opt_dev}
    ref = _engine(3, "fp32", 4, 3e-3)
    got = _engine(3, "fp32", 4, 3e-3, extra)
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-4), (got, ref)


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_partitioned_path_on_one_gpu(stage, monkeypatch):
    """The multi-GPU code path (RCCL all-gather on the ag stream, reduce-scatter on the rs stream, shard pointing,
    prefetch) forced on with a single rank: must still track torch.optim.AdamW."""
    monkeypatch.setenv("DS_ZERO_FORCE_PARTITION", "1")
    ref = _torch_ref(6, 3e-3)
    got = _engine(stage, "fp32", 6, 3e-3, {"stage3_param_persistence_threshold": 0})
    assert got == pytest.approx(ref, rel=2e-3, abs=2e-3), (got, ref)


def test_partitioned_zeropp_on_one_gpu(monkeypatch):
    """ZeRO++ qwZ (int8 weight all-gather) + qgZ (quantized gradient reduce-scatter) through the RCCL path."""
    monkeypatch.setenv("DS_ZERO_FORCE_PARTITION", "1")
    ref = _torch_ref(6, 3e-3)
    got = _engine(3, "bf16", 6, 3e-3, {"stage3_param_persistence_threshold": 0, "zero_quantized_weights": True,
                                       "zero_quantized_gradients": True})
    assert got == pytest.approx(ref, rel=5e-2, abs=5e-2), (got, ref)
