"""LR schedules against their closed forms (reference `tests/unit/runtime/test_lr_schedulers.py`)."""
import math

import pytest
import torch

from deepspeedsyclsupport_amd.runtime import lr_schedules as L


def _opt(lr=0.1):
    return torch.optim.SGD([torch.nn.Parameter(torch.zeros(2))], lr=lr)


def _lrs(sched, n):
    out = []
    for _ in range(n):
        sched.step()
        out.append(sched.get_last_lr()[0])
    return out


@pytest.mark.parametrize("wtype", ["log", "linear"])
def test_warmup_lr(wtype):
    s = L.WarmupLR(_opt(), warmup_min_lr=0.01, warmup_max_lr=0.1, warmup_num_steps=10, warmup_type=wtype)
    got = _lrs(s, 15)
    for it, lr in enumerate(got):
        g = (math.log(it + 1) / math.log(10) if wtype == "log" else it / 10) if it < 10 else 1.0
        assert lr == pytest.approx(0.01 + 0.09 * g)
    assert got[-1] == pytest.approx(0.1)


def test_warmup_decay_lr():
    s = L.WarmupDecayLR(_opt(), total_num_steps=30, warmup_min_lr=0.0, warmup_max_lr=0.1, warmup_num_steps=10,
                        warmup_type="linear")
    got = _lrs(s, 31)
    assert got[10] == pytest.approx(0.1) and got[20] == pytest.approx(0.05) and got[30] == pytest.approx(0.0)
    assert all(a >= b for a, b in zip(got[10:], got[11:]))


def test_warmup_cosine_lr():
    s = L.WarmupCosineLR(_opt(0.2), total_num_steps=20, warmup_min_ratio=0.1, warmup_num_steps=5, cos_min_ratio=0.01,
                         warmup_type="linear")
    got = _lrs(s, 20)
    assert got[0] == pytest.approx(0.2 * 0.1)
    real = 19 - 5 + 1
    want_last = 0.2 * (0.01 + 0.99 * 0.5 * (1 + math.cos(math.pi * real / 15)))
    assert got[-1] == pytest.approx(want_last)


def test_one_cycle_shape_and_momentum():
    opt = torch.optim.Adam([torch.nn.Parameter(torch.zeros(2))], lr=0.1)
    s = L.OneCycle(opt, cycle_min_lr=0.01, cycle_max_lr=0.1, cycle_first_step_size=10, cycle_momentum=True,
                   cycle_min_mom=0.8, cycle_max_mom=0.9, decay_lr_rate=0.5, decay_step_size=5)
    got = _lrs(s, 30)
    peak = max(range(len(got)), key=lambda i: got[i])
    assert got[peak] == pytest.approx(0.1) and 8 <= peak <= 10
    assert got[19] == pytest.approx(0.01, abs=1e-3)
    assert got[-1] < 0.01  # decay phase after the cycle
    assert opt.param_groups[0]["betas"][0] == pytest.approx(0.9, abs=1e-2)


def test_lr_range_test_and_state_dict():
    s = L.LRRangeTest(_opt(), lr_range_test_min_lr=0.01, lr_range_test_step_size=5, lr_range_test_step_rate=1.0,
                      lr_range_test_staircase=True)
    got = _lrs(s, 12)
    assert got[3] == pytest.approx(0.01) and got[4] == pytest.approx(0.02) and got[10] == pytest.approx(0.03)
    sd = s.state_dict()
    s2 = L.LRRangeTest(_opt(), lr_range_test_min_lr=0.01, lr_range_test_step_size=5, lr_range_test_staircase=True)
    s2.load_state_dict(sd)
    assert _lrs(s2, 1) == _lrs(s, 1)
