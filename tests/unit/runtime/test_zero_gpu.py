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


def _engine(stage, dtype, steps, lr, zero_extra=None, gas=1, split=False):
    import deepspeedsyclsupport_amd as ds
    from ..simple_model import base_config
    torch.manual_seed(0)
    m = tiny_llama(hidden_size=128, intermediate_size=256, num_attention_heads=4)
    cfg = base_config(stage=stage, lr=lr, mb=2, gas=gas, clip=1.0, dtype=dtype)
    cfg["zero_optimization"].update(zero_extra or {})
    if split:
        cfg["bf16"]["split_master_weights"] = True
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    out = []
    for x in _data(steps * gas, 5):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        out.append(float(loss))
    eng.optimizer.join_offload()
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


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("ratio", [1.0, 0.4])
def test_twin_flow_gpu_matches_device(ratio, overlap):
    """ZeRO-Offload (ratio 1) / Twin-Flow on the device path: gradients staged to pinned memory on the d2h stream
    during backward, native CPU Adam on the worker thread, weights back on the h2d stream — optionally with the next
    forward overlapping the host step — must match the all-device optimizer."""
    ref = _engine(3, "fp32", 5, 3e-3)
    got = _engine(3, "fp32", 5, 3e-3, {"offload_optimizer": {"device": "cpu", "ratio": ratio, "pin_memory": True,
                                                             "overlap_forward": overlap}})
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-4), (got, ref)


def test_three_tier_offload_gpu(tmp_path):
    """device + host DRAM + NVMe tail of optimizer state in one run, stepped through the pinned chunk pipeline."""
    ref = _engine(3, "fp32", 4, 3e-3)
    got = _engine(3, "fp32", 4, 3e-3, {"sub_group_size": 16384, "offload_optimizer": {
        "device": "nvme", "ratio": 0.7, "max_in_cpu": 150000, "nvme_path": str(tmp_path), "pin_memory": True}})
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-4), (got, ref)


@pytest.mark.parametrize("stage", [2, 3])
def test_offload_gradient_accumulation_partitioned_gpu(stage, monkeypatch):
    """gas 2 on the partitioned path: reduce-scattered segments go down through the bounce buffers into the fp32
    host accumulator."""
    monkeypatch.setenv("DS_ZERO_FORCE_PARTITION", "1")
    ref = _engine(stage, "fp32", 3, 3e-3, {"stage3_param_persistence_threshold": 0}, gas=2)
    got = _engine(stage, "fp32", 3, 3e-3, {"stage3_param_persistence_threshold": 0,
                                           "offload_optimizer": {"device": "cpu", "ratio": 0.6, "pin_memory": True}},
                  gas=2)
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-4), (got, ref)


@pytest.mark.parametrize("offload", [None, {"device": "cpu", "ratio": 0.5, "pin_memory": True}])
def test_split_master_weights_gpu(offload):
    """bf16 weight + int16 residual masters (fused split Adam kernel on the device, split CPU Adam on the host)
    follow the fp32-master bf16 run."""
    ref = _engine(3, "bf16", 6, 3e-3)
    extra = {"offload_optimizer": offload} if offload else None
    got = _engine(3, "bf16", 6, 3e-3, extra, split=True)
    assert got == pytest.approx(ref, rel=2e-2, abs=2e-2), (got, ref)


def test_split_adam_kernel_matches_fp32_master():
    """adam_multi_split tracks adam_multi on an fp32 master: join(hi, lo) follows the fp32 master step after step
    (to the last fp32 bits: the two kernels are separate compilations of the same arithmetic), on vector-aligned
    and odd-sized tensors, and the bf16 half is the master rounded to nearest."""
    from deepspeedsyclsupport_amd.ops.native import hip_ops
    from deepspeedsyclsupport_amd.runtime.zero.offload import split_cut, split_join
    torch.manual_seed(0)
    sizes = [8 * 4096 * 3, 1001]
    ps = [(torch.randn(n, device="cuda") * 0.05) for n in sizes]
    his, los = zip(*[split_cut(p) for p in ps])
    his, los = [h.clone() for h in his], [l.clone() for l in los]
    ms, vs = [torch.zeros_like(p) for p in ps], [torch.zeros_like(p) for p in ps]
    ms2, vs2 = [torch.zeros_like(p) for p in ps], [torch.zeros_like(p) for p in ps]
    for step in range(1, 5):
        gs = [(torch.randn_like(p) * 1e-2).bfloat16() for p in ps]
        lps = [torch.empty_like(p, dtype=torch.bfloat16) for p in ps]
        bc1, bc2 = 1 - 0.9**step, 1 - 0.95**step
        hip_ops().adam_multi(ps, ms, vs, gs, lps, 1e-2, 0.9, 0.95, 1e-8, 0.1, bc1, bc2, 0.5, True)
        hip_ops().adam_multi_split(los, ms2, vs2, gs, his, 1e-2, 0.9, 0.95, 1e-8, 0.1, bc1, bc2, 0.5, True)
        for p, hi, lo, m, m2 in zip(ps, his, los, ms, ms2):
            j = split_join(hi, lo)
            torch.testing.assert_close(j, p, rtol=1e-5, atol=2e-8)
            torch.testing.assert_close(m2, m, rtol=1e-5, atol=1e-10)
            assert bool(((hi.float() - j).abs() <= j.abs() * 2.0**-8).all())


@pytest.mark.parametrize("pdev", [None, "cpu"])
def test_frozen_parameters_partitioned_on_one_gpu(pdev, monkeypatch):
    """A frozen base (embedding, attention and norms of layer 0) with the rest trained, on the partitioned device
    path: frozen weights are fetched on the all-gather stream, released by the module backward hook, optionally homed
    in pinned host memory, and the trained ones follow plain PyTorch with the same parameters frozen."""
    import deepspeedsyclsupport_amd as ds
    from ..simple_model import base_config
    monkeypatch.setenv("DS_ZERO_FORCE_PARTITION", "1")

    def frozen_of(m):
        return [p for n, p in m.named_parameters() if "embed_tokens" in n or "layers.0.self_attn" in n
                or "layers.0.input_layernorm" in n]

    torch.manual_seed(0)
    ref_m = tiny_llama(hidden_size=128, intermediate_size=256, num_attention_heads=4).cuda()
    for p in frozen_of(ref_m):
        p.requires_grad_(False)
    opt = torch.optim.AdamW([p for p in ref_m.parameters() if p.requires_grad], lr=3e-3, weight_decay=0.01)
    ref = []
    for x in _data(5, 5):
        loss = ref_m(x, labels=x)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_([p for p in ref_m.parameters() if p.requires_grad], 1.0)
        opt.step()
        ref.append(float(loss))

    torch.manual_seed(0)
    m = tiny_llama(hidden_size=128, intermediate_size=256, num_attention_heads=4)
    for p in frozen_of(m):
        p.requires_grad_(False)
    before = [p.detach().clone() for p in frozen_of(m)]
    cfg = base_config(stage=3, lr=3e-3, mb=2, clip=1.0, dtype="fp32")
    cfg["zero_optimization"]["stage3_param_persistence_threshold"] = 0
    if pdev:
        cfg["zero_optimization"]["offload_param"] = {"device": pdev, "pin_memory": True}
    eng, *_ = ds.initialize(model=m, config=cfg, model_parameters=[p for p in m.parameters() if p.requires_grad])
    assert eng.optimizer.frozen_groups and all(g.partition for g in eng.optimizer.frozen_groups)
    got = []
    for x in _data(5, 5):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        got.append(float(loss))
    assert got == pytest.approx(ref, rel=2e-3, abs=2e-3), (got, ref)
    assert all(p.numel() == 0 for p in m.parameters())
    with ds.zero.GatheredParameters(frozen_of(m)):
        for p, b in zip(frozen_of(m), before):
            assert torch.equal(p.detach().cpu(), b)
