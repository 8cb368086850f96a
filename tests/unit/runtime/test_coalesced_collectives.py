"""`runtime/comm/coalesced_collectives` (reference `tests/unit/runtime/comm/test_coalesced_collectives.py`): one
batched reduce-scatter hands every rank the group average of its chunk of every tensor, also when sizes do not divide
the world size; the quantised variant follows it within int8 noise."""
import math

import torch

from ..common import run_distributed


def _run(out):
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.comm.coalesced_collectives import (all_to_all_quant_reduce,
                                                                            reduce_scatter_coalesced)
    dist.init_distributed("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    shapes = [(7, ), (64, ), (5, 3), (1, ), (130, )]
    mine = [torch.arange(math.prod(s), dtype=torch.float32).reshape(s) * (rank + 1) + i for i, s in enumerate(shapes)]
    parts = reduce_scatter_coalesced([t.clone() for t in mine])
    single = reduce_scatter_coalesced([mine[1].clone()])[0]  # the in-place wire-layout case
    big = torch.randn(world * 256, 8, generator=torch.Generator().manual_seed(rank))
    q = all_to_all_quant_reduce([big.clone(), mine[0].clone()])
    got = [None] * world
    dist.all_gather_object(got, {"parts": parts, "single": single, "q": q, "big": big})
    if rank == 0:
        torch.save({"got": got, "shapes": shapes}, out)


def test_reduce_scatter_coalesced_and_quantised(tmp_path):
    world = 3
    out = str(tmp_path / "r.pt")
    run_distributed(_run, world, out)
    r = torch.load(out)
    shapes = r["shapes"]
    for i, s in enumerate(shapes):
        n = math.prod(s)
        avg = sum(torch.arange(n, dtype=torch.float32) * (k + 1) + i for k in range(world)) / world
        chunk = math.ceil(n / world)
        rebuilt = torch.cat([r["got"][k]["parts"][i] for k in range(world)])
        assert rebuilt.numel() == n and torch.allclose(rebuilt, avg), (i, s)
        for k in range(world):
            assert r["got"][k]["parts"][i].numel() == max(0, min(chunk, n - k * chunk))
    avg1 = sum(torch.arange(64, dtype=torch.float32) * (k + 1) + 1 for k in range(world)) / world
    assert torch.allclose(torch.cat([r["got"][k]["single"] for k in range(world)]), avg1)
    big_avg = sum(r["got"][k]["big"] for k in range(world)).reshape(-1) / world
    qbig = torch.cat([r["got"][k]["q"][0] for k in range(world)])
    assert (qbig - big_avg).abs().max() < 0.05 and not torch.equal(qbig, big_avg)
    q1 = torch.cat([r["got"][k]["q"][1] for k in range(world)])
    assert torch.allclose(q1, sum(torch.arange(7, dtype=torch.float32) * (k + 1) for k in range(world)) / world)
