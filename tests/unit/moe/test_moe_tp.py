"""MoE next to tensor parallelism (reference `tests/unit/moe/test_moe_tp.py`, `moe/mappings.py`,
`utils/groups.py:179-290`): tokens duplicated over tensor-parallel ranks are dropped before the expert all-to-all and
gathered after it, so the layer computes what a single process computes; expert group rank lists follow the
reference's E+M+D example."""
import pytest
import torch
import torch.nn as nn

from ..common import run_distributed

H, E, S = 16, 4, 24


def _expert():
    return nn.Sequential(nn.Linear(H, 2 * H), nn.GELU(), nn.Linear(2 * H, H))


def _reference_layer():
    """Single-process oracle: gate + E whole experts, top-1 without token priority randomisation."""
    torch.manual_seed(0)
    gate = nn.Linear(H, E, bias=False)
    experts = [_expert() for _ in range(E)]
    return gate, experts


class _TPmpu:
    """Megatron-style mpu over `tp` consecutive ranks."""

    def __init__(self, tp):
        from deepspeedsyclsupport_amd import comm as dist
        self.tp = tp
        world, rank = dist.get_world_size(), dist.get_rank()
        self.tp_group = self.dp_group = None
        for i in range(world // tp):
            ranks = list(range(i * tp, (i + 1) * tp))
            g = dist.new_group(ranks)
            if rank in ranks:
                self.tp_group = g
        for i in range(tp):
            ranks = list(range(i, world, tp))
            g = dist.new_group(ranks)
            if rank in ranks:
                self.dp_group = g
        self.rank, self.world = rank, world

    def get_tensor_model_parallel_world_size(self):
        return self.tp

    def get_tensor_model_parallel_rank(self):
        return self.rank % self.tp

    def get_tensor_model_parallel_group(self):
        return self.tp_group

    get_model_parallel_world_size = get_tensor_model_parallel_world_size
    get_model_parallel_rank = get_tensor_model_parallel_rank
    get_model_parallel_group = get_tensor_model_parallel_group

    def get_data_parallel_world_size(self):
        return self.world // self.tp

    def get_data_parallel_rank(self):
        return self.rank // self.tp

    def get_data_parallel_group(self):
        return self.dp_group


def _run(tp, ep, drop, out):
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.moe.layer import MoE
    from deepspeedsyclsupport_amd.parallel import groups
    dist.init_distributed("gloo")
    groups.mpu = _TPmpu(tp)
    rank, world = dist.get_rank(), dist.get_world_size()
    gate, experts = _reference_layer()
    torch.manual_seed(1)
    moe = MoE(H, _expert(), num_experts=E, ep_size=ep, k=1, capacity_factor=2.0, min_capacity=2, use_rts=False,
              drop_tokens=drop)
    ep_rank = groups._get_expert_parallel_rank(moe.expert_group_name)
    with torch.no_grad():
        moe.deepspeed_moe.gate.wg.weight.copy_(gate.weight)
        L = E // ep
        for l, e in enumerate(moe.deepspeed_moe.experts.deepspeed_experts):
            e.load_state_dict(experts[ep_rank * L + l].state_dict())
    # every tensor-parallel rank of a replica sees the same tokens; replicas see different ones
    g = torch.Generator().manual_seed(10 + rank // tp)
    x = torch.randn(S, H, generator=g, requires_grad=True)
    y, l_aux, _ = moe(x)
    y.square().sum().backward()
    # oracle on this replica's tokens
    xr = x.detach().clone().requires_grad_(True)
    gates = torch.softmax(gate(xr.float()), dim=1)
    idx = gates.argmax(1)
    cap = moe.deepspeed_moe.gate.min_capacity
    import math
    cap = max(math.ceil(S / E * 2.0), 2) if drop else None
    ref = torch.zeros_like(xr)
    rows = []
    for e in range(E):
        tok = (idx == e).nonzero().flatten()
        if cap is not None:
            c = -(-cap // tp) * tp
            tok = tok[:c]
        if tok.numel():
            rows.append((tok, experts[e](xr[tok]) * gates[tok, e:e + 1]))
    ref = torch.zeros(S, H).index_add(0, torch.cat([t for t, _ in rows]), torch.cat([v for _, v in rows]))
    ref.square().sum().backward()
    res = dict(err=float((y - ref).abs().max()), gerr=float((x.grad - xr.grad).abs().max()),
               ref=float(ref.abs().max()))
    got = [None] * world
    dist.all_gather_object(got, res)
    if rank == 0:
        torch.save(got, out)


@pytest.mark.parametrize("world,tp,ep,drop", [(2, 2, 2, True), (4, 2, 2, True), (4, 2, 4, False)])
def test_moe_with_tensor_parallel_non_experts(world, tp, ep, drop, tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_run, world, tp, ep, drop, out)
    for r in torch.load(out):
        assert r["ref"] > 1e-3
        assert r["err"] < 1e-5 and r["gerr"] < 1e-4, r


def test_expert_parallel_rank_lists():
    from deepspeedsyclsupport_amd.parallel.groups import _get_expert_parallel_ranks
    ep, edp = _get_expert_parallel_ranks(16, 2, 4)
    assert ep == [[0, 2, 4, 6], [8, 10, 12, 14], [1, 3, 5, 7], [9, 11, 13, 15]]
    assert edp == [[0, 8], [2, 10], [4, 12], [6, 14], [1, 9], [3, 11], [5, 13], [7, 15]]
    ep, edp = _get_expert_parallel_ranks(32, 2, 4, use_data_before_expert_parallel_=True)
    assert ep[0] == [0, 8, 16, 24] and len(ep) == 8 and sorted(sum(ep, [])) == list(range(32))
    assert all(len(g) == 4 for g in edp) and sorted(sum(edp, [])) == list(range(32))
