"""ZeRO-3 fetch / gather / release event counters (reference `runtime/zero/partitioned_param_profiler.py`).

The coordinator reports every event with the elements it moved; with wall-clock timers (`wall_clock_breakdown`)
the host time of each event kind is kept too. `log_events()` prints count, elements and (if timed) milliseconds per
event kind; the engine calls it every `steps_per_print` steps. Device-side timing of the same phases comes from the
roctx ranges (`rocprofv3 --marker-trace`, `tools/gpu_prof_markers.sh`)."""
from dataclasses import dataclass

from ...utils.logging import log_dist

FETCH, ALLGATHER, PREFETCH, RELEASE, REUSE = "fetch", "all_gather", "prefetch", "release", "reuse_hit"


class PartitionedParameterProfiler:

    @dataclass
    class EventCounter:
        name: str
        count: int = 0
        num_elem: int = 0

        def reset(self):
            self.count = 0
            self.num_elem = 0

        def increment(self, numel):
            self.count += 1
            self.num_elem += numel

    def __init__(self, timers=None):
        self.timers = timers
        self.event_counters = {}

    def reset_events(self):
        for c in self.event_counters.values():
            c.reset()

    def start_event(self, name):
        self.event_counters.setdefault(name, self.EventCounter(name))
        if self.timers is not None:
            self.timers(name).start()

    def stop_event(self, name, num_elem):
        self.event_counters.setdefault(name, self.EventCounter(name)).increment(int(num_elem))
        if self.timers is not None:
            self.timers(name).stop()

    def count(self, name, num_elem):
        self.event_counters.setdefault(name, self.EventCounter(name)).increment(int(num_elem))

    def summary(self):
        return {n: (c.count, c.num_elem) for n, c in self.event_counters.items()}

    def log_events(self):
        for c in self.event_counters.values():
            line = f"ZeRO-3 {c.name}: count = {c.count}, numel = {c.num_elem}"
            if self.timers is not None and c.name in getattr(self.timers, "timers", {}):
                line += f", {self.timers(c.name).elapsed(reset=True):.2f} ms"
            log_dist(line, ranks=[0])
