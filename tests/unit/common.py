"""Multi-process test harness (reference `tests/unit/common.py:105-368` DistributedExec/DistributedTest).

`run_distributed(fn, world_size, *args)` forks `world_size` ranks, sets RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* (127.0.0.1,
free port), initialises torch.distributed (gloo on the host, nccl=RCCL when `backend="nccl"`), runs `fn(*args)` in
every rank and re-raises the first failure (with its traceback) in the parent. Skips propagate.
"""
import multiprocessing as mp
import os
import socket
import traceback

import pytest

DEFAULT_TIMEOUT = int(os.environ.get("DS_TEST_TIMEOUT", "300"))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, backend, fn, args, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "gloo":
        os.environ["DS_ACCELERATOR"] = "cpu"
    try:
        import deepspeedsyclsupport_amd as ds
        ds.init_distributed(dist_backend=backend)
        from deepspeedsyclsupport_amd.parallel import groups
        groups.reset()
        fn(*args)
        q.put((rank, "ok", ""))
    except pytest.skip.Exception as e:
        q.put((rank, "skip", str(e)))
    except BaseException:
        q.put((rank, "fail", traceback.format_exc()))
    finally:
        try:
            import torch.distributed as tdist
            if tdist.is_initialized():
                tdist.destroy_process_group()
        except Exception:
            pass


_CTX = None


def _context(backend):
    # forkserver (not fork): the pytest parent has already spun up torch/OpenMP thread pools, and forking a process
    # with live thread pools can deadlock the children. The server preloads torch + the package once, so ranks start
    # fast anyway (reference harness uses forkserver too, `tests/unit/common.py:148`).
    global _CTX
    if _CTX is None:
        _CTX = mp.get_context("forkserver")
        _CTX.set_forkserver_preload(["torch", "deepspeedsyclsupport_amd"])
    return _CTX


def run_distributed(fn, world_size=2, *args, backend="gloo", timeout=DEFAULT_TIMEOUT):
    ctx = _context(backend)
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, backend, fn, args, q)) for r in range(world_size)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in range(world_size):
            results.append(q.get(timeout=timeout))
    except Exception:
        for p in procs:
            p.kill()
        raise TimeoutError(f"distributed test timed out after {timeout}s")
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    fails = [r for r in results if r[1] == "fail"]
    if fails:
        raise AssertionError("\n".join(f"[rank {r}] {tb}" for r, _, tb in fails))
    skips = [r for r in results if r[1] == "skip"]
    if skips:
        pytest.skip(skips[0][2])
