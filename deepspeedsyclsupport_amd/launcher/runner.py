"""`deepspeed` CLI: resource discovery + multi-node fan-out (reference `launcher/runner.py:388-597`).

Same user contract as the reference: a hostfile of `host slots=N` lines, `--include/--exclude` filters in
`NODE[:SLOT,SLOT][@NODE...]` syntax, `--num_nodes/--num_gpus`, a base64 world-info blob handed to the per-node
launcher (`launcher.launch`), and pdsh / OpenMPI / MPICH / Intel-MPI / Slurm / MVAPICH runners for multi-node.
MI355X specifics: local GPUs are counted without initialising HIP (`torch.cuda.device_count()` only reads the
driver), and the per-node launcher exports `HIP_VISIBLE_DEVICES` plus `HSA_ENABLE_IPC_MODE_LEGACY=0` (dmabuf IPC,
required for RCCL over xGMI on these hosts).
"""
import argparse
import base64
import collections
import json
import os
import re
import subprocess
import sys

from ..utils.logging import logger
from .constants import (DEFAULT_HOSTFILE, EXPORT_ENVS, MPICH_LAUNCHER, MVAPICH_LAUNCHER, OPENMPI_LAUNCHER,
                        PDSH_LAUNCHER, SLURM_LAUNCHER, IMPI_LAUNCHER, TORCH_DISTRIBUTED_DEFAULT_PORT)

DEEPSPEED_ENVIRONMENT_NAME = os.getenv("DS_ENV_FILE", ".deepspeed_env")
DEEPSPEED_ENVIRONMENT_PATHS = [os.path.expanduser("~"), "."]


def parse_args(args=None):
    p = argparse.ArgumentParser(description="DeepSpeed (MI355X) distributed launcher")
    p.add_argument("-H", "--hostfile", type=str, default=DEFAULT_HOSTFILE)
    p.add_argument("-i", "--include", type=str, default="")
    p.add_argument("-e", "--exclude", type=str, default="")
    p.add_argument("--num_nodes", type=int, default=-1)
    p.add_argument("--min_elastic_nodes", type=int, default=-1)
    p.add_argument("--max_elastic_nodes", type=int, default=-1)
    p.add_argument("--num_gpus", "--num_accelerators", type=int, default=-1)
    p.add_argument("--master_port", type=int, default=TORCH_DISTRIBUTED_DEFAULT_PORT)
    p.add_argument("--master_addr", type=str, default="")
    p.add_argument("--launcher", type=str, default=PDSH_LAUNCHER)
    p.add_argument("--launcher_args", type=str, default="")
    p.add_argument("--module", action="store_true")
    p.add_argument("--no_python", action="store_true")
    p.add_argument("--no_local_rank", action="store_true")
    p.add_argument("--no_ssh_check", action="store_true")
    p.add_argument("--force_multi", action="store_true")
    p.add_argument("--save_pid", action="store_true")
    p.add_argument("--enable_each_rank_log", type=str, default="None")
    p.add_argument("--autotuning", type=str, default="", choices=["", "tune", "run"])
    p.add_argument("--elastic_training", action="store_true")
    p.add_argument("--bind_cores_to_rank", action="store_true")
    p.add_argument("--bind_core_list", type=str, default=None)
    p.add_argument("--ssh_port", type=int, default=None)
    p.add_argument("user_script", type=str)
    p.add_argument("user_args", nargs=argparse.REMAINDER)
    return p.parse_args(args=args)


# ------------------------------------------------------------------------------------------------ hostfile
_HOST_RE = re.compile(r"^(\S+)\s+slots=(\d+)\s*$")


def parse_hostfile_lines(lines):
    """`host slots=N` per line, '#' comments; returns OrderedDict host -> slots."""
    pool = collections.OrderedDict()
    for raw in lines:
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        m = _HOST_RE.match(line)
        if not m:
            raise ValueError(f"Hostfile contains a bad entry: {line!r}")
        host, slots = m.group(1), int(m.group(2))
        if host in pool:
            raise ValueError(f"Hostfile contains multiple entries for {host}")
        pool[host] = slots
    if not pool:
        raise ValueError("Hostfile is empty or not formatted correctly")
    return pool


def fetch_hostfile(path):
    if not os.path.isfile(path):
        logger.warning("Unable to find hostfile, will proceed with training with local resources only.")
        return None
    with open(path) as f:
        return parse_hostfile_lines(f.readlines())


def _spec_items(spec):
    """'a@b:0,2' -> [('a', None), ('b', [0, 2])]"""
    out = []
    for node in spec.split("@"):
        if ":" in node:
            host, slots = node.split(":", 1)
            out.append((host, [int(s) for s in slots.split(",") if s != ""]))
        else:
            out.append((node, None))
    return out


def parse_resource_filter(host_info, include_str="", exclude_str=""):
    """Filter {host: [slots]} by an include OR exclude spec (mutually exclusive); preserves hostfile order."""
    if include_str and exclude_str:
        raise ValueError("include_str and exclude_str are mutually exclusive.")
    if not include_str and not exclude_str:
        return host_info
    chosen = {} if include_str else {h: list(s) for h, s in host_info.items()}
    for host, slots in _spec_items(include_str or exclude_str):
        if host not in host_info:
            raise ValueError(f"Hostname '{host}' not found in hostfile")
        for s in slots or []:
            if s not in host_info[host]:
                raise ValueError(f"No slot '{s}' specified on host '{host}'")
        if include_str:
            prev = chosen.get(host, [])
            add = host_info[host] if slots is None else slots
            chosen[host] = prev + [s for s in add if s not in prev]
        else:
            chosen[host] = [] if slots is None else [s for s in chosen[host] if s not in slots]
    return collections.OrderedDict((h, chosen[h]) for h in host_info if chosen.get(h))


def parse_inclusion_exclusion(resource_pool, inclusion, exclusion):
    active = collections.OrderedDict((h, list(range(n))) for h, n in resource_pool.items())
    return parse_resource_filter(active, include_str=inclusion, exclude_str=exclusion)


def parse_num_nodes(str_num_nodes: str, elastic_training: bool):
    """`--num_nodes` as (min, max): "4" -> (4, -1); "2:8" (elastic training only) -> (2, 8)."""
    parts = str(str_num_nodes).split(":")
    if len(parts) == 1:
        return int(parts[0]), -1
    if len(parts) == 2 and elastic_training:
        lo, hi = int(parts[0]), int(parts[1])
        if lo < 1 or hi < lo:
            raise RuntimeError("MIN:MAX format of num_nodes needs 1 <= MIN <= MAX")
        return lo, hi
    if len(parts) == 2:
        raise RuntimeError("MIN:MAX format is only supported in elastic training")
    raise RuntimeError(f"num_nodes {str_num_nodes} is not in MIN:MAX format")


def encode_world_info(world_info):
    return base64.urlsafe_b64encode(json.dumps(world_info).encode("utf-8")).decode("utf-8")


def decode_world_info(blob):
    return json.loads(base64.urlsafe_b64decode(blob))


def _local_gpu_count():
    try:
        import torch
        return torch.cuda.device_count()  # reads the driver only; does not initialise HIP
    except Exception:
        return 0


def build_active_resources(args):
    pool = fetch_hostfile(args.hostfile)
    multi = pool is not None
    if pool is None:
        if args.include or args.exclude:
            raise ValueError("include/exclude require a hostfile")
        n = args.num_gpus if args.num_gpus > 0 else max(_local_gpu_count(), 1)
        pool = collections.OrderedDict(localhost=n)
    active = parse_inclusion_exclusion(pool, args.include, args.exclude)
    if args.num_nodes > 0:
        active = collections.OrderedDict(list(active.items())[:args.num_nodes])
    if args.num_gpus > 0:
        active = collections.OrderedDict((h, s[:args.num_gpus]) for h, s in active.items())
    return active, multi


def _load_env_file():
    exports = {}
    for d in DEEPSPEED_ENVIRONMENT_PATHS:
        f = os.path.join(d, DEEPSPEED_ENVIRONMENT_NAME)
        if os.path.isfile(f):
            with open(f) as fh:
                for line in fh:
                    line = line.strip()
                    if line and not line.startswith("#") and "=" in line:
                        k, v = line.split("=", 1)
                        exports[k] = v
    return exports


def main(args=None):
    args = parse_args(args)
    active, multi = build_active_resources(args)
    if not active:
        raise RuntimeError("no resources left after include/exclude filtering")
    if not args.master_addr:
        args.master_addr = next(iter(active)) if multi else "127.0.0.1"
    if args.autotuning:
        from ..autotuning import Autotuner
        tuner = Autotuner(args, active)
        best = tuner.tune()
        tuner.print_tuning_results()
        if args.autotuning == "tune" or best is None:
            return 0
        # "run": launch the user script with the optimal config
        opt_cfg = os.path.join(tuner.results_dir, "ds_config_optimal.json")
        ua = list(args.user_args)
        if "--deepspeed_config" in ua:
            ua[ua.index("--deepspeed_config") + 1] = opt_cfg
        args.user_args = ua
        args.autotuning = ""
    world_info = encode_world_info(active)
    multi_node = args.force_multi or len(active) > 1
    if args.elastic_training:
        assert not args.no_local_rank, "--no_local_rank is not supported with elastic training"

    if not multi_node:
        cmd = [sys.executable, "-u", "-m", "deepspeedsyclsupport_amd.launcher.launch", f"--world_info={world_info}",
               f"--master_addr={args.master_addr}", f"--master_port={args.master_port}"]
        for flag in ("no_python", "no_local_rank", "module", "save_pid", "bind_cores_to_rank"):
            if getattr(args, flag):
                cmd.append(f"--{flag}")
        if args.enable_each_rank_log != "None":
            cmd.append(f"--enable_each_rank_log={args.enable_each_rank_log}")
        if args.bind_core_list:
            cmd.append(f"--bind_core_list={args.bind_core_list}")
        cmd += [args.user_script] + args.user_args
        env = os.environ.copy()
        env.update(_load_env_file())
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    else:
        from .multinode_runner import RUNNERS
        runner_cls = RUNNERS.get(args.launcher.lower())
        if runner_cls is None:
            raise NotImplementedError(f"Unknown launcher {args.launcher}")
        runner = runner_cls(args, world_info, active)
        if not runner.backend_exists():
            raise RuntimeError(f"launcher '{args.launcher}' not installed")
        env = os.environ.copy()
        for k, v in env.items():
            if any(k.startswith(p) for p in EXPORT_ENVS):
                runner.add_export(k, v)
        for k, v in _load_env_file().items():
            runner.add_export(k, v)
        runner.add_export("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = runner.get_cmd(env, active)
    logger.info(f"cmd = {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, env=env)
    rc = proc.wait()
    if rc != 0:
        sys.exit(rc)
    return rc


if __name__ == "__main__":
    main()
