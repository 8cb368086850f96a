"""Elastic worker-group supervisor (reference `elasticity/elastic_agent.py:28-181` `DSElasticAgent`, a
torch-elastic `LocalElasticAgent` subclass started by `launcher/launch.py --enable_elastic_training`).

One agent per node starts the node's ranks as child processes, then monitors them. When any rank fails (non-zero
exit, killed, or silent past `heartbeat_timeout` when a heartbeat file is configured) the agent stops the whole
group and restarts it — up to `max_restarts` times — on a fresh rendezvous port, exporting the restart count as
`TORCHELASTIC_RESTART_COUNT` (the same variable torch-elastic uses) so the training script resumes from its latest
checkpoint. A clean exit of every rank ends the run. Restarting the group on the same world size mirrors the
reference's behaviour on a single node (membership changes need a multi-node rendezvous the reference delegates to
torch-elastic's c10d backend); `compute_elastic_config` keeps the global batch valid when the world size differs
between attempts.

Failure injection for testing recovery lives in `utils/fault_injection.py` (`DS_FAULT_INJECT`).
"""
import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..utils.logging import logger


def _free_port(addr="127.0.0.1"):
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


@dataclass
class WorkerSpec:
    cmd: List[str]                               # argv of one rank (the same for every rank)
    nproc: int                                   # ranks on this node
    env: Dict[str, str] = field(default_factory=dict)
    node_rank: int = 0
    nnodes: int = 1
    master_addr: str = "127.0.0.1"
    master_port: Optional[int] = None
    max_restarts: int = 3
    monitor_interval: float = 0.5
    log_dir: Optional[str] = None
    heartbeat_dir: Optional[str] = None          # ranks touch <dir>/rank<r>; silence > heartbeat_timeout = hang
    heartbeat_timeout: float = 0.0
    rank_offset: Optional[int] = None             # global rank of this node's local rank 0 (default node_rank*nproc)
    world_size: Optional[int] = None              # default nproc * nnodes


@dataclass
class RunResult:
    state: str                                   # "SUCCEEDED" | "FAILED"
    restarts: int
    return_codes: Dict[int, int]


class DSElasticAgent:

    def __init__(self, spec: WorkerSpec, env: Optional[Dict[str, str]] = None):
        self.spec = spec
        self.ds_env = dict(env or {})
        self.remaining_restarts = spec.max_restarts
        self.procs: List[subprocess.Popen] = []
        self._logs = []

    # ------------------------------------------------------------------------------------------ workers
    def _start_workers(self, attempt):
        s = self.spec
        port = s.master_port if (s.master_port and attempt == 0) else _free_port(s.master_addr)
        world = s.world_size or s.nproc * s.nnodes
        base = s.rank_offset if s.rank_offset is not None else s.node_rank * s.nproc
        self.procs, self._logs = [], []
        for lr in range(s.nproc):
            rank = base + lr
            env = os.environ.copy()
            env.update(self.ds_env)
            env.update(s.env)
            env.update({
                "RANK": str(rank), "LOCAL_RANK": str(lr), "WORLD_SIZE": str(world), "LOCAL_WORLD_SIZE": str(s.nproc),
                "GROUP_RANK": str(s.node_rank), "MASTER_ADDR": s.master_addr, "MASTER_PORT": str(port),
                "TORCHELASTIC_RESTART_COUNT": str(attempt), "TORCHELASTIC_MAX_RESTARTS": str(s.max_restarts),
                "HSA_ENABLE_IPC_MODE_LEGACY": "0",
            })
            if s.heartbeat_dir:
                env["DS_HEARTBEAT_FILE"] = os.path.join(s.heartbeat_dir, f"rank{rank}")
            out = None
            if s.log_dir:
                d = os.path.join(s.log_dir, f"attempt_{attempt}")
                os.makedirs(d, exist_ok=True)
                out = open(os.path.join(d, f"rank{rank}.log"), "w")
                self._logs.append(out)
            # own process group per rank so a hung rank and its children can be stopped as a unit
            self.procs.append(subprocess.Popen(s.cmd, env=env, stdout=out, stderr=subprocess.STDOUT if out else None,
                                               start_new_session=True))
        self._started = time.time()
        logger.info(f"elastic agent: attempt {attempt} started {s.nproc} ranks on port {port}")

    def _stop_workers(self, grace=10.0):
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + grace
        for p in self.procs:
            try:
                p.wait(timeout=max(deadline - time.time(), 0.1))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
        for f in self._logs:
            f.close()
        self._logs = []

    def _hung_ranks(self):
        s = self.spec
        if not s.heartbeat_dir or s.heartbeat_timeout <= 0:
            return []
        now, hung = time.time(), []
        for lr, p in enumerate(self.procs):
            if p.poll() is not None:
                continue
            base = s.rank_offset if s.rank_offset is not None else s.node_rank * s.nproc
            f = os.path.join(s.heartbeat_dir, f"rank{base + lr}")
            last = os.path.getmtime(f) if os.path.exists(f) else self._started
            if now - max(last, self._started) > s.heartbeat_timeout:
                hung.append(lr)
        return hung

    def _monitor(self):
        """-> ("SUCCEEDED"|"FAILED"|"HEALTHY", return codes)."""
        codes = {i: p.poll() for i, p in enumerate(self.procs)}
        if any(c not in (None, 0) for c in codes.values()):
            return "FAILED", codes
        if self._hung_ranks():
            return "FAILED", codes
        if all(c == 0 for c in codes.values()):
            return "SUCCEEDED", codes
        return "HEALTHY", codes

    # ------------------------------------------------------------------------------------------ run loop
    def run(self) -> RunResult:
        attempt = 0
        self._start_workers(attempt)
        try:
            while True:
                time.sleep(self.spec.monitor_interval)
                state, codes = self._monitor()
                if state == "SUCCEEDED":
                    return RunResult("SUCCEEDED", attempt, {k: v for k, v in codes.items()})
                if state == "FAILED":
                    bad = {k: v for k, v in codes.items() if v not in (None, 0)}
                    logger.warning(f"elastic agent: worker group failed (exit codes {bad}, hung "
                                   f"{self._hung_ranks()}); {self.remaining_restarts} restarts left")
                    self._stop_workers()
                    if self.remaining_restarts <= 0:
                        return RunResult("FAILED", attempt, {k: (v if v is not None else -9) for k, v in codes.items()})
                    self.remaining_restarts -= 1
                    attempt += 1
                    self._start_workers(attempt)
        finally:
            self._stop_workers()


def main(argv=None):
    """`python -m deepspeedsyclsupport_amd.elasticity.elastic_agent --nproc N --max_restarts R -- cmd ...`"""
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("--max_restarts", type=int, default=3)
    ap.add_argument("--master_addr", default="127.0.0.1")
    ap.add_argument("--master_port", type=int, default=None)
    ap.add_argument("--log_dir", default=None)
    ap.add_argument("--heartbeat_timeout", type=float, default=0.0)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    hb = None
    if a.heartbeat_timeout > 0:
        import tempfile
        hb = tempfile.mkdtemp(prefix="ds_hb_")
    res = DSElasticAgent(WorkerSpec(cmd=cmd, nproc=a.nproc, master_addr=a.master_addr, master_port=a.master_port,
                                    max_restarts=a.max_restarts, log_dir=a.log_dir, heartbeat_dir=hb,
                                    heartbeat_timeout=a.heartbeat_timeout)).run()
    logger.info(f"elastic agent: {res.state} after {res.restarts} restarts")
    return 0 if res.state == "SUCCEEDED" else 1


if __name__ == "__main__":
    sys.exit(main())
