"""FLOPs profiler, timers and the comms logger (reference `tests/unit/profiling/flops_profiler/test_flops_profiler.py`,
`utils/timer.py`, `tests/unit/comm/test_dist.py` comms logging)."""
import time

import torch
import torch.nn as nn

from ..common import run_distributed


class MLP(nn.Module):

    def __init__(self, d=32, h=64):
        super().__init__()
        self.fc1 = nn.Linear(d, h)
        self.fc2 = nn.Linear(h, d)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


def test_get_model_profile_counts_matmul_flops():
    from deepspeedsyclsupport_amd.profiling.flops_profiler import get_model_profile
    m = MLP()
    flops, macs, params = get_model_profile(m, input_shape=(4, 32), print_profile=False, as_string=False)
    # two linears: 2 * batch * in * out each (bias adds and ReLU are not matmul-class work)
    assert flops == 2 * 4 * 32 * 64 * 2 and macs == flops / 2
    assert params == sum(p.numel() for p in m.parameters())


def test_profiler_start_stop_and_report(tmp_path):
    from deepspeedsyclsupport_amd.profiling.flops_profiler import FlopsProfiler
    m = MLP()
    prof = FlopsProfiler(m)
    prof.start_profile()
    m(torch.randn(8, 32))
    prof.stop_profile()
    assert prof.get_total_flops() == 2 * 8 * 32 * 64 * 2
    assert prof.get_total_duration() > 0
    out = tmp_path / "prof.txt"
    prof.print_model_profile(output_file=str(out))
    prof.end_profile()
    text = out.read_text()
    assert "fc1" in text or "MLP" in text


def test_timers():
    from deepspeedsyclsupport_amd.utils.timer import SynchronizedWallClockTimer, ThroughputTimer
    t = SynchronizedWallClockTimer()
    t("fwd").start()
    time.sleep(0.01)
    t("fwd").stop()
    assert t("fwd").elapsed(reset=False) >= 5.0  # milliseconds
    logged = []
    tp = ThroughputTimer(batch_size=16, start_step=1, steps_per_output=2, logging_fn=logged.append)
    for _ in range(5):
        tp.start()
        time.sleep(0.002)
        tp.stop(global_step=True)
    assert tp.avg_samples_per_sec() > 0 and logged


def _comms(out):
    from deepspeedsyclsupport_amd import comm as dist
    dist.configure(enabled=True, prof_all=True, verbose=False)
    x = torch.ones(1024)
    for _ in range(3):
        dist.all_reduce(x)
    y = torch.empty(2048)
    dist.all_gather_into_tensor(y, torch.ones(1024))
    if dist.get_rank() == 0:
        s = dist.comms_logger.log_all(print_log=False)
        torch.save({"summary": s, "ops": sorted(dist.comms_logger.comms_dict)}, out)


def test_comms_logger_records_ops(tmp_path):
    out = str(tmp_path / "c.pt")
    run_distributed(_comms, 2, out)
    d = torch.load(out, weights_only=True)
    assert any("all_reduce" in o for o in d["ops"]) and any("all_gather" in o for o in d["ops"])
    assert "busbw" in d["summary"]
