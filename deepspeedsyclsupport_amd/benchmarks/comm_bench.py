"""Collective-communication benchmark behind `ds_bench` (reference `benchmarks/communication/{run_all,all_reduce,
all_gather,all_to_all,broadcast,pt2pt}.py` + `bin/ds_bench`).

One process per GPU (launched by torch.distributed.run on 127.0.0.1 when started without the launcher env), RCCL
over xGMI on device tensors; every op is timed over a size sweep with CUDA events after warm-up, and rank 0 prints
size, latency, algorithm bandwidth and bus bandwidth (the reference's busbw conventions, `comm/comms_logging.py`)
plus the per-xGMI-link figure (busbw / (world - 1): on a fully connected node every peer pair has its own link).
`inference_all_reduce` times the native peer-mapped small-message path (`comm/xgmi.py`).
"""
import argparse
import json
import os
import sys

import torch

OPS = ("all_reduce", "all_gather", "reduce_scatter", "all_to_all", "broadcast", "pt2pt", "inference_all_reduce")


def parser():
    p = argparse.ArgumentParser(prog="ds_bench", description=__doc__.split("\n\n")[0])
    p.add_argument("--ops", default="all_reduce,all_gather,reduce_scatter,all_to_all,broadcast",
                   help=f"comma list of {OPS}")
    p.add_argument("--minsize", type=int, default=1 << 12, help="smallest message in bytes")
    p.add_argument("--maxsize", type=int, default=1 << 30, help="largest message in bytes")
    p.add_argument("--trials", type=int, default=20)
    p.add_argument("--warmups", type=int, default=5)
    p.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float16", "float32"])
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--nproc", type=int, default=0, help="ranks to launch when not started by a launcher (0 = #GPUs)")
    p.add_argument("--json", default=None, help="also write the rows here (rank 0)")
    p.add_argument("--local_rank", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    return p


def bus_factor(op, n):
    if op in ("all_reduce", "inference_all_reduce"):
        return 2 * (n - 1) / n
    if op in ("all_gather", "reduce_scatter", "all_to_all"):
        return (n - 1) / n
    return 1.0


def _timed(fn, trials, warmups, device):
    for _ in range(warmups):
        fn()
    if device.type == "cuda":
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(trials):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / 1e3 / trials
    import time
    t = time.perf_counter()
    for _ in range(trials):
        fn()
    return (time.perf_counter() - t) / trials


def run(args):
    import torch.distributed as tdist
    from .. import comm as dist
    dist.init_distributed(dist_backend=args.backend, verbose=False)
    rank, n = tdist.get_rank(), tdist.get_world_size()
    device = torch.device("cuda", torch.cuda.current_device()) if args.backend == "nccl" else torch.device("cpu")
    dtype = getattr(torch, args.dtype)
    es = torch.tensor([], dtype=dtype).element_size()
    rows = []
    for op in args.ops.split(","):
        if op not in OPS:
            raise SystemExit(f"unknown op {op}; choose from {OPS}")
        size = args.minsize
        while size <= args.maxsize:
            numel = max(n * 8, size // es // (n * 8) * (n * 8))  # divisible by the world (and 16 B per rank)
            x = torch.ones(numel, dtype=dtype, device=device)
            if op == "all_reduce":
                fn = lambda: tdist.all_reduce(x)  # noqa: E731
            elif op == "inference_all_reduce":
                fn = lambda: dist.inference_all_reduce(x)  # noqa: E731
            elif op == "all_gather":
                out = torch.empty(numel * n, dtype=dtype, device=device)
                fn = lambda: tdist.all_gather_into_tensor(out, x)  # noqa: E731
            elif op == "reduce_scatter":
                out = torch.empty(numel // n, dtype=dtype, device=device)
                fn = lambda: tdist.reduce_scatter_tensor(out, x)  # noqa: E731
            elif op == "all_to_all":
                out = torch.empty_like(x)
                fn = lambda: tdist.all_to_all_single(out, x)  # noqa: E731
            elif op == "broadcast":
                fn = lambda: tdist.broadcast(x, 0)  # noqa: E731
            else:  # pt2pt: ranks 0 <-> 1 ping-pong, the others idle
                def fn():
                    if rank == 0:
                        tdist.send(x, 1)
                        tdist.recv(x, 1)
                    elif rank == 1:
                        tdist.recv(x, 0)
                        tdist.send(x, 0)
            tdist.barrier()
            t = _timed(fn, args.trials, args.warmups, device)
            tt = torch.tensor([t], device=device)
            tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
            t = float(tt)
            nbytes = numel * es * (n if op == "all_gather" else 1)
            if op == "pt2pt":
                t /= 2
            algbw = nbytes / t / 1e9
            busbw = algbw * bus_factor(op, n)
            row = {"op": op, "bytes": nbytes, "world": n, "latency_us": round(t * 1e6, 2),
                   "algbw_GBps": round(algbw, 4), "busbw_GBps": round(busbw, 4),
                   "per_link_GBps": round(busbw / max(n - 1, 1), 4) if op != "pt2pt" else round(algbw, 4)}
            rows.append(row)
            if rank == 0:
                print(json.dumps(row), flush=True)
            size *= 4
    if rank == 0 and args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)
    tdist.barrier()
    tdist.destroy_process_group()
    return rows


def main(argv=None):
    argv = list(argv if argv is not None else sys.argv[1:])
    if "DS_BENCH_ARGV" in os.environ:  # re-launched child: the arguments travel outside the launcher's parser
        argv = json.loads(os.environ["DS_BENCH_ARGV"])
    args = parser().parse_args(argv)
    if all(k in os.environ for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")):
        run(args)
        return 0
    # not under a launcher: start one rank per GPU on this node and exit with its status
    import socket
    import subprocess
    nproc = args.nproc or max(torch.cuda.device_count(), 1)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "deepspeedsyclsupport_amd.benchmarks.comm_bench"]
    env = dict(os.environ, DS_BENCH_ARGV=json.dumps(argv))
    env["PYTHONPATH"] = os.pathsep.join([os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))] +
                                        [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p])
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())
