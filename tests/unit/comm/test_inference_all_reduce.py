"""`comm.inference_all_reduce` fast paths (comm/xgmi.py): POSIX-shm reduce for host tensors (CPU, gloo ranks) and
the peer-mapped xGMI kernel for device tensors (GPU: two ranks sharing the box's one GPU, gloo for the handle
exchange — the kernel, the IPC mapping and the flag protocol are the same as across GPUs)."""
import pytest
import torch

from ..common import run_distributed


def _shm_run(sizes):
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.comm import xgmi
    rank, world = dist.get_rank(), dist.get_world_size()
    for it in range(3):
        for n in sizes:
            for dt in (torch.float32, torch.bfloat16):
                g = torch.Generator().manual_seed(1000 * it + n)
                base = torch.randn(world, n, generator=g)
                t = base[rank].to(dt).clone()
                dist.inference_all_reduce(t)
                ref = base.to(dt).float().sum(0)
                tol = 1e-5 if dt == torch.float32 else 3e-2
                torch.testing.assert_close(t.float(), ref, rtol=tol, atol=tol * world)
    assert xgmi._shm.get(0) is not None, "host tensors must take the shm path"
    if world == 4:  # two disjoint groups -> two segments
        g0, g1 = dist.new_group([0, 1]), dist.new_group([2, 3])
        mine = g0 if rank < 2 else g1
        t = torch.full((1000, ), float(rank + 1))
        dist.inference_all_reduce(t, group=mine)
        assert torch.all(t == (3.0 if rank < 2 else 7.0))
    xgmi.reset()


@pytest.mark.parametrize("world", [2, 4])
def test_shm_inference_all_reduce(world):
    run_distributed(_shm_run, world, [8, 1000, 70001, 1 << 20 + 3])


def _xgmi_run():
    import os
    from deepspeedsyclsupport_amd.comm.xgmi import XgmiAllReduce
    from deepspeedsyclsupport_amd import comm as dist
    if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") not in (None, "0"):
        pytest.skip("needs dmabuf IPC")
    torch.cuda.set_device(0)
    rank, world = dist.get_rank(), dist.get_world_size()
    ar = XgmiAllReduce(None, cap_bytes=4 << 20)
    for it in range(4):
        for n in (8, 4096 * 8, 65536, 1 << 20):
            for dt in (torch.bfloat16, torch.float32, torch.float16):
                if n * torch.tensor([], dtype=dt).element_size() > ar.cap:
                    continue
                for mode in (1, 2):
                    g = torch.Generator().manual_seed(7 * it + n + mode)
                    base = torch.randn(world, n, generator=g)
                    t = base[rank].to(dt).cuda()
                    out = torch.empty_like(t) if mode == 2 else None
                    y = ar.all_reduce(t, out=out, mode=mode)
                    ref = base.to(dt).float().sum(0)
                    tol = 1e-5 if dt == torch.float32 else 2e-2
                    torch.testing.assert_close(y.float().cpu(), ref, rtol=tol, atol=tol * world)
    # HIP-graph capture: the epoch lives on the device, so replays keep the protocol in step
    x = torch.zeros(8192, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ar.all_reduce(x, mode=1)
    for k in range(3):
        x.fill_(float(rank + k))
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        assert torch.all(x.float() == float(sum(r + k for r in range(world)))), (k, x[:4])
    assert ar.error() == 0
    dist.barrier()
    ar.close()


@pytest.mark.gpu
def test_xgmi_all_reduce_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    run_distributed(_xgmi_run, 2, timeout=240)


def _xgmi_timeout_run():
    """A peer that arrives later than the wait limit: the waiting rank's kernel leaves on its own (bounded wait),
    its output is all NaN (never a partial sum), the next call raises until the error word is reset, and after the
    reset the two ranks are still in step. The condition is forced from the host (one rank sleeps before launching,
    the other has a 20 ms limit); every kernel exits normally."""
    import os
    import time
    from deepspeedsyclsupport_amd.comm.xgmi import XgmiAllReduce
    from deepspeedsyclsupport_amd import comm as dist
    if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") not in (None, "0"):
        pytest.skip("needs dmabuf IPC")
    torch.cuda.set_device(0)
    rank, world = dist.get_rank(), dist.get_world_size()
    ar = XgmiAllReduce(None, cap_bytes=1 << 20)
    x = torch.full((4096, ), float(rank + 1), dtype=torch.float32, device="cuda")
    ar.all_reduce(x, mode=1)
    torch.cuda.synchronize()
    assert torch.all(x == 3.0) and ar.error() == 0
    dist.barrier()
    if rank == 0:
        ar.set_timeout_ms(20.0)
    else:
        time.sleep(1.0)  # the straggler
    y = torch.full((4096, ), float(rank + 1), dtype=torch.float32, device="cuda")
    ar.all_reduce(y, mode=1)
    torch.cuda.synchronize()
    if rank == 0:
        assert bool(torch.isnan(y).all()), y[:4]
        assert ar.error() == 2  # 1 + index of the peer that was late
        with pytest.raises(RuntimeError, match="did not arrive"):
            ar.all_reduce(y, mode=1)
        assert ar.error(reset=True) == 2 and ar.error() == 0
        ar.set_timeout_ms(5000.0)
    else:
        assert torch.all(y == 3.0)  # the late rank found its peer's data and flag already there
    dist.barrier()
    z = torch.full((4096, ), float(rank + 1), dtype=torch.float32, device="cuda")
    ar.all_reduce(z, mode=2)
    torch.cuda.synchronize()
    assert torch.all(z == 3.0), z[:4]
    dist.barrier()
    ar.close()


@pytest.mark.gpu
def test_xgmi_all_reduce_timeout_is_loud():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    run_distributed(_xgmi_timeout_run, 2, timeout=240)
