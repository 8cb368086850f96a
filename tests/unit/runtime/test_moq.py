"""MoQ quantize-in-optimizer-step, eigenvalue-stretched bit schedule and progressive layer drop through the engine
(reference `tests/unit/runtime/quantize/*`, `tests/unit/runtime/test_pld.py`; `runtime/quantize.py`,
`runtime/engine.py:1384-1401,2069-2079`)."""
import math

import pytest
import torch
import torch.nn as nn

from deepspeedsyclsupport_amd.runtime.quantize import Quantizer

from ..common import run_distributed


def _param(shape, start, target, period, seed=0):
    torch.manual_seed(seed)
    p = nn.Parameter(torch.randn(*shape))
    p.start_bits, p.target_bits, p.q_period = start, target, period
    return p


def test_highbit_symmetric_levels_and_error():
    q = Quantizer(q_groups=4, q_type="symmetric", q_rounding="nearest")
    p = _param((8, 32), 6, 6, 100)
    out = q.compute_quantization(p)
    for row in out.reshape(4, -1):
        assert row.unique().numel() <= 2**6
    # error bounded by half a step of each group's grid, except the group's +max, which the reference grid
    # [-2^(b-1), 2^(b-1) - 1] clamps one step down
    x = p.data.reshape(4, -1)
    step = 2 * x.abs().amax(1, keepdim=True) / 2**6
    err = (out.reshape(4, -1) - x).abs()
    assert (err <= step + 1e-6).all()
    assert (err[x < x.amax(1, keepdim=True)] <= (step / 2 + 1e-6).expand_as(x)[x < x.amax(1, keepdim=True)]).all()


def test_highbit_asymmetric_zero_point():
    q = Quantizer(q_groups=1, q_type="asymmetric", q_rounding="nearest")
    p = _param((4, 16), 4, 4, 100)
    p.data.add_(3.0)  # all positive: an asymmetric grid covers [min, max] only
    out = q.compute_quantization(p)
    assert out.unique().numel() <= 16
    step = (p.data.max() - p.data.min()) / 16
    assert (out - p.data).abs().max() <= step + 1e-5


def test_ternary_and_binary():
    q = Quantizer(q_groups=2, q_type="symmetric", q_rounding="nearest")
    t = q.quantize_tenary(torch.randn(4, 8))
    for row in t.reshape(2, -1):
        assert row.abs().unique().numel() <= 2  # {0, alpha}
    b = q.quantize_binary(torch.randn(4, 8))
    for row in b.reshape(2, -1):
        assert row.abs().unique().numel() == 1 and row.abs()[0] > 0


def test_bit_schedule_period_doubles():
    q = Quantizer(q_groups=1)
    p = _param((4, 8), 8, 5, 2)
    seen = []
    for _ in range(16):
        q.quantize([[p]], overflow=False, eigenvalue_enabled=False)
        seen.append((q.qsteps, p.start_bits, p.q_period))
    # drops at step 2 (period -> 4), 4 (-> 8), 8 (-> 16); stops at the target
    assert [s for s in seen if s[0] in (1, 2, 4, 8, 16)] == [(1, 8, 2), (2, 7, 4), (4, 6, 8), (8, 5, 16),
                                                            (16, 5, 16)]


def test_eigenvalue_factor_stretches_period():
    q = Quantizer(q_groups=1, q_eigenvalue=True, layer_num=1)
    p = _param((4, 8), 8, 4, 1)
    q.quantize([[p]], overflow=False, eigenvalue_enabled=True, block_eigenvalue={id(p): (0.6, 0)})
    assert p.start_bits == 7 and p.q_period == (1 << 1) * (1 + math.floor(0.6 * 4))


def test_mixed_fp16_ratio_blends():
    q = Quantizer(q_groups=1, q_mixed_fp16=True, q_change_ratio=0.25)
    p = _param((4, 8), 4, 4, 100)
    w = p.data.clone()
    out = q.compute_quantization(p)  # ratio 1.0: still the real weights
    torch.testing.assert_close(out, w)
    q.update_fp16_ratio()
    q.update_fp16_ratio()
    out = q.compute_quantization(p)
    pure = Quantizer(q_groups=1).quantize_highbit(w, 4)
    torch.testing.assert_close(out, 0.5 * w + 0.5 * pure)


def test_overflow_skips_without_eigenvalue():
    q = Quantizer()
    p = _param((4, 8), 8, 8, 10)
    w = p.data.clone()
    q.quantize([[p]], overflow=True, eigenvalue_enabled=False)
    assert q.qsteps == 0 and torch.equal(p.data, w)


class _Block(nn.Module):

    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(16, 16)

    def forward(self, x):
        return x + torch.tanh(self.fc(x))


class _Net(nn.Module):

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.layers = nn.ModuleList([_Block() for _ in range(2)])
        self.head = nn.Linear(16, 4)
        self.seen = []

    def forward(self, x, y, progressive_layer_drop=False, pld_theta=1.0):
        self.seen.append((progressive_layer_drop, pld_theta))
        for l in self.layers:
            x = l(x)
        return nn.functional.cross_entropy(self.head(x), y)


def _moq_engine(eigen):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.compression import init_compression
    cfg = {"train_batch_size": 4, "train_micro_batch_size_per_gpu": 4,
           "optimizer": {"type": "Adam", "params": {"lr": 1e-2}},
           "progressive_layer_drop": {"enabled": True, "theta": 0.5, "gamma": 0.1},
           "compression_training": {"weight_quantization": {
               "shared_parameters": {"enabled": True, "quantize_weight_in_forward": False, "quantize_groups": 2,
                                     "schedule_offset": 0, "quantization_type": "symmetric",
                                     "rounding": "nearest"},
               "different_groups": {"wq": {"params": {"start_bits": 8, "target_bits": 6, "quantization_period": 2},
                                           "modules": ["layers.*"]}}}}}
    if eigen:
        cfg["eigenvalue"] = {"enabled": True, "max_iter": 5, "tol": 1e-2, "layer_name": "layers", "layer_num": 2,
                             "gas_boundary_resolution": 1}
    net = _Net()
    init_compression(net, cfg)
    engine, *_ = ds.initialize(model=net, model_parameters=net.parameters(), config=cfg)
    torch.manual_seed(1)
    x, y = torch.randn(4, 16), torch.randint(0, 4, (4, ))
    for _ in range(3):
        loss = engine(x, y)
        engine.backward(loss)
        engine.step()
    w = engine.module.layers[0].fc.weight
    # quantize() ran before the first forward and after each of the 3 steps: 8 -> 7 bits at qstep 2 (period 2 -> 4),
    # 7 -> 6 (the target) at qstep 4 (period -> 8); the weights sit on the 6-bit grid of each group
    assert engine.quantizer is not None and engine.quantizer.qsteps == 4
    # (with eigenvalues every new period is also multiplied by 1 + floor(4 * eigenvalue) of the weight's block, so
    # after the first drop the next one is still ahead)
    bits = w.start_bits
    if eigen:
        ev = engine.block_eigenvalue[id(w)][0]
        assert bits == 7 and w.q_period == 4 * (1 + math.floor(4 * ev))
    else:
        assert (bits, w.q_period) == (6, 8)
    for row in w.detach().reshape(2, -1):
        assert row.unique().numel() <= 2**bits
    # the head is not a compress layer: untouched by MoQ
    assert not hasattr(engine.module.head.weight, "start_bits")
    # PLD: the forward got the keep probability, decaying from 1 towards theta
    thetas = [t for (on, t) in net.seen if on]
    assert len(thetas) == 3 and thetas[0] == 1.0 and thetas[-1] < 1.0
    if eigen:
        assert engine.block_eigenvalue is not None and id(w) in engine.block_eigenvalue


@pytest.mark.parametrize("eigen", [False, True])
def test_engine_moq_and_pld(eigen):
    run_distributed(_moq_engine, 1, eigen)
