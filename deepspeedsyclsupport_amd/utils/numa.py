"""NUMA helpers for the launcher (reference `utils/numa.py`): parse `numactl --hardware`, split the node's cores
between the local ranks and build the `numactl` prefix that binds each rank to its share."""
import os
import shutil
import subprocess


def get_numa_cores():
    """[[core ids of NUMA node 0], [node 1], ...] (empty list when numactl is unavailable)."""
    if shutil.which("numactl") is None:
        return []
    out = subprocess.check_output(["numactl", "--hardware"]).decode()
    cores = []
    for line in out.splitlines():
        parts = line.split()
        if len(parts) > 3 and parts[0] == "node" and parts[2] == "cpus:":
            cores.append([int(c) for c in parts[3:]])
    return cores


def check_for_numactl_pkg():
    return shutil.which("numactl") is not None


def parse_range(rng):
    lo, _, hi = rng.partition("-")
    return list(range(int(lo), int(hi or lo) + 1))


def parse_range_list(range_str):
    """'0-3,8,10-11' -> sorted unique core ids."""
    out = set()
    for part in range_str.split(","):
        if part:
            out.update(parse_range(part))
    return sorted(out)


def get_numactl_cmd(bind_core_list, num_local_procs, local_rank):
    """-> (cores per rank, ['numactl', ...] prefix). Cores are split evenly; a rank whose cores all sit on one NUMA
    node also gets `-m <node>` (memory binding), otherwise `-l` (local allocation)."""
    cores = parse_range_list(bind_core_list) if bind_core_list else list(range(os.cpu_count() or 1))
    per_rank = len(cores) // num_local_procs
    if per_rank == 0:
        raise ValueError(f"{len(cores)} cores cannot be split between {num_local_procs} ranks")
    mine = cores[local_rank * per_rank:(local_rank + 1) * per_rank]
    cmd = ["numactl"]
    nodes = get_numa_cores()
    on = [n for n, cs in enumerate(nodes) if set(mine) <= set(cs)]
    cmd += ["-m", str(on[0])] if on else ["-l"]
    cmd += ["-C", ",".join(str(c) for c in mine)]
    return per_rank, cmd
