"""Per-node process launcher (reference `launcher/launch.py:132-355`).

Spawns one process per local GPU slot with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_SIZE / CROSS_RANK / CROSS_SIZE /
MASTER_ADDR / MASTER_PORT, restricts each node to its slots with HIP_VISIBLE_DEVICES, optionally pins every rank
to a core range with numactl (`--bind_cores_to_rank`), writes per-rank logs, and tears the whole node down when
any rank fails (so a hung collective never outlives a crashed peer).
"""
import argparse
import os
import shutil
import signal
import subprocess
import sys
import time

from ..utils.logging import logger
from .runner import decode_world_info

PID_FILE_BASEPATH = "/tmp"


def parse_args(args=None):
    p = argparse.ArgumentParser()
    p.add_argument("--node_rank", type=int, default=-1)
    p.add_argument("--master_addr", default="127.0.0.1", type=str)
    p.add_argument("--master_port", default=29500, type=int)
    p.add_argument("--world_info", default="None", type=str)
    p.add_argument("--module", action="store_true")
    p.add_argument("--no_python", action="store_true")
    p.add_argument("--enable_elastic_training", action="store_true")
    p.add_argument("--min_elastic_nodes", type=int, default=-1)
    p.add_argument("--max_elastic_nodes", type=int, default=-1)
    p.add_argument("--max_restarts", type=int, default=3, help="elastic: worker-group restarts before giving up")
    p.add_argument("--heartbeat_timeout", type=float, default=0.0,
                   help="elastic: restart the group when a rank's step heartbeat is older than this (s)")
    p.add_argument("--no_local_rank", action="store_true")
    p.add_argument("--save_pid", type=int, default=0, nargs="?", const=1)
    p.add_argument("--enable_each_rank_log", default="None", type=str)
    p.add_argument("--bind_cores_to_rank", action="store_true")
    p.add_argument("--bind_core_list", type=str, default=None)
    p.add_argument("training_script", type=str)
    p.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return p.parse_args(args=args)


def _node_rank(args, hosts):
    if args.node_rank >= 0:
        return args.node_rank
    for var in ("OMPI_COMM_WORLD_NODE_RANK", "SLURM_NODEID", "PMI_NODE_RANK", "NODE_RANK"):
        if var in os.environ:
            return int(os.environ[var])
    import socket
    name = socket.gethostname()
    for i, h in enumerate(hosts):
        if h in (name, name.split(".")[0]):
            return i
    return 0


def _core_ranges(n_local, core_list=None):
    cores = core_list if core_list is not None else list(range(os.cpu_count() or 1))
    per = max(len(cores) // max(n_local, 1), 1)
    return [cores[i * per:(i + 1) * per] for i in range(n_local)]


def parse_core_list(spec):
    out = []
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def terminate_process_tree(pid):
    """SIGTERM a process and all its descendants; SIGKILL whatever is still alive after 30 s."""
    import psutil
    try:
        root = psutil.Process(pid)
    except psutil.NoSuchProcess:
        return
    procs = root.children(recursive=True) + [root]
    for p in procs:
        try:
            p.terminate()
        except psutil.NoSuchProcess:
            pass
    _, alive = psutil.wait_procs(procs, timeout=30)
    for p in alive:
        try:
            p.kill()
        except psutil.NoSuchProcess:
            pass


def build_rank_envs(world_info, node_rank, master_addr, master_port):
    """Per-local-rank environment dicts for this node (pure; unit-tested)."""
    hosts = list(world_info.keys())
    host = hosts[node_rank]
    slots = world_info[host]
    offsets, acc = [], 0
    for h in hosts:
        offsets.append(acc)
        acc += len(world_info[h])
    world = acc
    envs = []
    for local_rank, _ in enumerate(slots):
        envs.append({
            "RANK": str(offsets[node_rank] + local_rank),
            "LOCAL_RANK": str(local_rank),
            "WORLD_SIZE": str(world),
            "LOCAL_SIZE": str(len(slots)),
            "CROSS_RANK": str(node_rank),
            "CROSS_SIZE": str(len(hosts)),
            "MASTER_ADDR": master_addr,
            "MASTER_PORT": str(master_port),
            "HIP_VISIBLE_DEVICES": ",".join(str(s) for s in slots),
            "HSA_ENABLE_IPC_MODE_LEGACY": "0",
        })
    return envs


def main(args=None):
    args = parse_args(args)
    world_info = decode_world_info(args.world_info)
    hosts = list(world_info.keys())
    node_rank = _node_rank(args, hosts)
    envs = build_rank_envs(world_info, node_rank, args.master_addr, args.master_port)
    logger.info(f"node_rank={node_rank} local ranks={len(envs)} world={envs[0]['WORLD_SIZE'] if envs else 0}")
    numactl = shutil.which("numactl")
    cores = parse_core_list(args.bind_core_list) if args.bind_core_list else None
    ranges = _core_ranges(len(envs), cores)
    if args.enable_elastic_training:
        return _run_elastic(args, envs)
    procs, logs = [], []
    for local_rank, renv in enumerate(envs):
        env = os.environ.copy()
        env.update(renv)
        cmd = []
        if args.bind_cores_to_rank and numactl:
            r = ranges[local_rank]
            cmd += [numactl, f"--physcpubind={r[0]}-{r[-1]}"]
            env["OMP_NUM_THREADS"] = str(len(r))
        if not args.no_python:
            cmd += [sys.executable, "-u"]
            if args.module:
                cmd.append("-m")
        cmd.append(args.training_script)
        if not args.no_local_rank:
            cmd.append(f"--local_rank={local_rank}")
        cmd += args.training_script_args
        stdout = None
        if args.enable_each_rank_log != "None":
            os.makedirs(args.enable_each_rank_log, exist_ok=True)
            f = open(os.path.join(args.enable_each_rank_log, f"rank{renv['RANK']}.log"), "w")
            logs.append(f)
            stdout = f
        procs.append(subprocess.Popen(cmd, env=env, stdout=stdout, stderr=subprocess.STDOUT if stdout else None))
    if args.save_pid:
        with open(os.path.join(PID_FILE_BASEPATH, f"{os.getpid()}.deepspeed"), "w") as f:
            f.write(" ".join(str(p.pid) for p in procs))

    def _terminate(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 15
        for p in procs:
            try:
                p.wait(timeout=max(deadline - time.time(), 0.1))
            except subprocess.TimeoutExpired:
                p.kill()

    signal.signal(signal.SIGINT, lambda *a: (_terminate(), sys.exit(1)))
    signal.signal(signal.SIGTERM, lambda *a: (_terminate(), sys.exit(1)))
    rc = 0
    alive = set(range(len(procs)))
    while alive:
        for i in list(alive):
            code = procs[i].poll()
            if code is None:
                continue
            alive.discard(i)
            if code != 0:
                logger.error(f"rank {envs[i]['RANK']} exited with code {code}; terminating the node")
                rc = code
                _terminate()
                alive.clear()
                break
        time.sleep(0.2)
    for f in logs:
        f.close()
    return rc


def _run_elastic(args, envs):
    """Supervise this node's ranks with the elastic agent (restart the group on failure, `--max_restarts`)."""
    import tempfile
    from ..elasticity.elastic_agent import DSElasticAgent, WorkerSpec
    cmd = [] if args.no_python else [sys.executable, "-u"] + (["-m"] if args.module else [])
    cmd += [args.training_script] + args.training_script_args
    e0 = envs[0]
    world, nproc = int(e0["WORLD_SIZE"]), len(envs)
    common = {k: v for k, v in e0.items() if k not in ("RANK", "LOCAL_RANK")}
    hb = tempfile.mkdtemp(prefix="ds_hb_") if args.heartbeat_timeout > 0 else None
    spec = WorkerSpec(cmd=cmd, nproc=nproc, env=common, node_rank=int(e0.get("CROSS_RANK", 0)),
                      nnodes=int(e0.get("CROSS_SIZE", 1)), rank_offset=int(e0["RANK"]), world_size=world,
                      master_addr=e0["MASTER_ADDR"],
                      master_port=int(e0["MASTER_PORT"]), max_restarts=args.max_restarts,
                      log_dir=None if args.enable_each_rank_log == "None" else args.enable_each_rank_log,
                      heartbeat_dir=hb, heartbeat_timeout=args.heartbeat_timeout)
    res = DSElasticAgent(spec).run()
    logger.info(f"elastic run {res.state} after {res.restarts} restart(s)")
    return 0 if res.state == "SUCCEEDED" else 1


if __name__ == "__main__":
    sys.exit(main())
