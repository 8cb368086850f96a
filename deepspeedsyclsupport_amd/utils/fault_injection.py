"""Env-driven fault injection for recovery testing (SURVEY §5.3 design item; the reference has none).

`DS_FAULT_INJECT="rank=1,step=3,mode=exit[,attempt=0][,code=13]"` makes the given global rank fail when the engine
finishes optimizer step `step`, but only in restart attempt `attempt` (default 0, read from
TORCHELASTIC_RESTART_COUNT) so the restarted group runs through. Modes:
  exit  - os._exit(code) without cleanup (a crashed rank)
  raise - raise RuntimeError (a Python-level failure)
  hang  - stop making progress (sleep); a supervisor with a heartbeat timeout must detect it
  kill  - SIGKILL itself
Several faults can be given separated by ';'. Also refreshes the heartbeat file named by DS_HEARTBEAT_FILE each step.
"""
import os
import signal
import time


def _parse(spec):
    out = []
    for item in filter(None, (s.strip() for s in spec.split(";"))):
        kv = dict(p.split("=", 1) for p in item.split(","))
        out.append(dict(rank=int(kv.get("rank", 0)), step=int(kv.get("step", 1)), mode=kv.get("mode", "exit"),
                        attempt=int(kv.get("attempt", 0)), code=int(kv.get("code", 13))))
    return out


class FaultInjector:

    def __init__(self, rank):
        self.rank = rank
        self.faults = _parse(os.environ.get("DS_FAULT_INJECT", ""))
        self.attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        self.heartbeat = os.environ.get("DS_HEARTBEAT_FILE")

    @property
    def active(self):
        return bool(self.faults) or self.heartbeat is not None

    def on_step(self, global_step):
        if self.heartbeat:
            with open(self.heartbeat, "a"):
                os.utime(self.heartbeat, None)
        for f in self.faults:
            if f["rank"] == self.rank and f["step"] == global_step and f["attempt"] == self.attempt:
                mode = f["mode"]
                if mode == "exit":
                    os._exit(f["code"])
                if mode == "raise":
                    raise RuntimeError(f"injected fault at step {global_step} on rank {self.rank}")
                if mode == "kill":
                    os.kill(os.getpid(), signal.SIGKILL)
                if mode == "hang":
                    while True:
                        time.sleep(3600)
                raise ValueError(f"unknown fault mode {mode}")
