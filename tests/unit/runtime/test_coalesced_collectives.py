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


def _two_level(out_path):
    """4 ranks as 2 "nodes" of 2: the two-level quantised reduce-scatter against the exact sum, and against the
    single-level exchange's error."""
    import deepspeedsyclsupport_amd.comm as dist
    from deepspeedsyclsupport_amd.parallel import groups
    from deepspeedsyclsupport_amd.runtime.comm.coalesced_collectives import all_to_all_quant_reduce
    from deepspeedsyclsupport_amd.runtime.zero.zeropp import (quantized_reduce_scatter,
                                                             quantized_reduce_scatter_2level, swizzle_quant)
    from deepspeedsyclsupport_amd.ops.quantizer.quantizer import dequantize
    dist.init_distributed("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    table = groups._get_local_all_to_all_group(devices_per_node=2)
    assert set(table) == {"local_0", "local_1", "global_0", "global_1"}
    local, glob = table[f"local_{rank // 2}"], table[f"global_{rank % 2}"]
    seg = 512
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(world * seg, generator=g)
    every = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(every, x)
    exact = sum(e[rank * seg:(rank + 1) * seg] for e in every)
    out2 = torch.empty(seg)
    quantized_reduce_scatter_2level(out2, x, local, glob)
    out1 = torch.empty(seg)
    quantized_reduce_scatter(out1, x, None)
    scale = exact.abs().max()
    e2, e1 = (out2 - exact).abs().max() / scale, (out1 - exact).abs().max() / scale
    assert e2 < 0.03 and e1 < 0.03, (float(e1), float(e2))
    # the swizzle puts the chunks for local peer b first-to-last by node
    qt = swizzle_quant(torch.arange(4 * 64, dtype=torch.float32), 2, 2, 64)
    back = dequantize(qt, torch.float32).view(4, 64)
    assert [int(round(float(back[i, 0]) / 64)) for i in range(4)] == [0, 2, 1, 3]
    # the free function takes the reference's group table
    m = torch.randn(world * 64, 8, generator=g)
    got = all_to_all_quant_reduce([m], {**table, "world": None})[0]
    ms = [torch.empty_like(m) for _ in range(world)]
    dist.all_gather(ms, m)
    want = (sum(ms) / world).reshape(-1)[rank * 64 * 8:(rank + 1) * 64 * 8]
    assert (got.float() - want).abs().max() < 0.05 * want.abs().max() + 0.02
    if rank == 0:
        torch.save({"e1": float(e1), "e2": float(e2)}, out_path)


def test_two_level_quantized_reduce_scatter(tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_two_level, 4, out)
    r = torch.load(out, weights_only=True)
    assert r["e2"] < 0.03
