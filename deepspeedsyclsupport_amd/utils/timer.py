"""Wall-clock timers (reference `deepspeed/utils/timer.py:43-290`): event-based on HIP, host-based on CPU."""
import time

import torch

from ..accelerator import get_accelerator
from .logging import log_dist

FORWARD_MICRO_TIMER = "fwd_microstep"
FORWARD_GLOBAL_TIMER = "fwd"
BACKWARD_MICRO_TIMER = "bwd_microstep"
BACKWARD_GLOBAL_TIMER = "bwd"
BACKWARD_INNER_MICRO_TIMER = "bwd_inner_microstep"
BACKWARD_INNER_GLOBAL_TIMER = "bwd_inner"
BACKWARD_REDUCE_MICRO_TIMER = "bwd_allreduce_microstep"
BACKWARD_REDUCE_GLOBAL_TIMER = "bwd_allreduce"
STEP_MICRO_TIMER = "step_microstep"
STEP_GLOBAL_TIMER = "step"


class _Timer:

    def __init__(self, name):
        self.name_ = name
        self.started_ = False
        self.elapsed_records = []
        self._host = get_accelerator().use_host_timers()
        self._t0 = None
        self._ev = None

    def start(self):
        assert not self.started_, f"{self.name_} timer has already been started"
        if self._host:
            self._t0 = time.perf_counter()
        else:
            self._ev = get_accelerator().Event(enable_timing=True)
            self._ev.record()
        self.started_ = True

    def stop(self, reset=False, record=False):
        assert self.started_, "timer is not started"
        if self._host:
            self.elapsed_records.append((self._t0, time.perf_counter()))
        else:
            end = get_accelerator().Event(enable_timing=True)
            end.record()
            self.elapsed_records.append((self._ev, end))
        self.started_ = False

    def _resolve(self):
        out = 0.0
        for a, b in self.elapsed_records:
            if self._host:
                out += (b - a) * 1e3
            else:
                b.synchronize()
                out += a.elapsed_time(b)
        return out

    def reset(self):
        self.started_ = False
        self.elapsed_records = []

    def elapsed(self, reset=True):
        started = self.started_
        if started:
            self.stop()
        ms = self._resolve()
        if reset:
            self.reset()
        if started:
            self.start()
        return ms

    def mean(self):
        n = max(len(self.elapsed_records), 1)
        return self.elapsed(reset=False) / n


class SynchronizedWallClockTimer:
    """Group of named timers; `log()` prints averaged ms across ranks."""

    def __init__(self):
        self.timers = {}

    def get_timers(self):
        return self.timers

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name)
        return self.timers[name]

    @staticmethod
    def memory_usage():
        acc = get_accelerator()
        return (f" | mem_allocated: {acc.memory_allocated() / 2**30:.4f} GB"
                f" | max_mem_allocated: {acc.max_memory_allocated() / 2**30:.4f} GB")

    def log(self, names, normalizer=1.0, reset=True, memory_breakdown=False, ranks=None):
        assert normalizer > 0.0
        s = "time (ms)"
        for n in names:
            if n in self.timers:
                s += f" | {n}: {self.timers[n].elapsed(reset=reset) / normalizer:.2f}"
        if memory_breakdown:
            s += self.memory_usage()
        log_dist(s, ranks=ranks or [0])

    def get_mean(self, names, normalizer=1.0, reset=True):
        return {n: self.timers[n].mean() / normalizer for n in names if n in self.timers}


class NoopTimer:

    class Timer:

        def start(self):
            pass

        def reset(self):
            pass

        def stop(self, **kw):
            pass

        def elapsed(self, **kw):
            return 0

        def mean(self):
            return 0

    def __init__(self):
        self.timer = self.Timer()

    def __call__(self, name):
        return self.timer

    def get_timers(self):
        return {}

    def log(self, *a, **k):
        pass

    def get_mean(self, *a, **k):
        return {}


class ThroughputTimer:
    """Samples/sec (and tokens/sec if seq_length given) over global steps (reference `timer.py:198-290`)."""

    def __init__(self, batch_size, start_step=2, steps_per_output=50, monitor_memory=False, logging_fn=None,
                 seq_length=None):
        self.batch_size = max(batch_size, 1)
        self.start_step = start_step
        self.steps_per_output = steps_per_output
        self.logging = logging_fn or (lambda m: log_dist(m, ranks=[0]))
        self.seq_length = seq_length
        self.global_step_count = 0
        self.micro_step_count = 0
        self.total_elapsed_time = 0.0
        self.step_elapsed_time = 0.0
        self.started = False
        self._t = None

    def update_epoch_count(self):
        pass

    def start(self):
        self.started = True
        if self.global_step_count >= self.start_step:
            get_accelerator().synchronize()
            self._t = time.time()

    def stop(self, global_step=False, report_speed=True):
        if not self.started:
            return
        self.started = False
        self.micro_step_count += 1
        if global_step:
            self.global_step_count += 1
        if self._t is not None:
            get_accelerator().synchronize()
            dt = time.time() - self._t
            self._t = None
            self.total_elapsed_time += dt
            self.step_elapsed_time += dt
            if global_step and report_speed and self.global_step_count % self.steps_per_output == 0:
                msg = f"epoch=0/micro_step={self.micro_step_count}/global_step={self.global_step_count}, " \
                      f"RunningAvgSamplesPerSec={self.avg_samples_per_sec():.3f}, " \
                      f"CurrSamplesPerSec={self.batch_size * self.steps_per_output / max(self.step_elapsed_time, 1e-9):.3f}"
                self.logging(msg)
                self.step_elapsed_time = 0.0

    def avg_samples_per_sec(self):
        steps = self.global_step_count - self.start_step
        if steps > 0 and self.total_elapsed_time > 0:
            return self.batch_size * steps / self.total_elapsed_time
        return float("-inf")


class CudaEventTimer:
    """Elapsed time between two recorded device events (HIP events here), in milliseconds."""

    def __init__(self, start_event, end_event):
        self.start_event = start_event
        self.end_event = end_event

    def get_elapsed_msec(self):
        get_accelerator().current_stream().wait_event(self.end_event)
        self.end_event.synchronize()
        return self.start_event.elapsed_time(self.end_event)


def trim_mean(data, trim_percent):
    """Mean of `data` after dropping the `trim_percent` smallest and largest fraction of the values."""
    assert 0.0 <= trim_percent <= 1.0
    n = len(data)
    if n == 0:
        return 0
    data = sorted(data)
    k = int(round(n * trim_percent))
    kept = data[k:n - k] or data
    return sum(kept) / len(kept)

