"""Pipeline parallelism (reference `tests/unit/runtime/pipe/test_pipe.py`): 1F1B over gloo vs single process."""
import pytest
import torch
import torch.nn as nn

from ..common import run_distributed

H, L, M, MB, STEPS = 16, 6, 4, 2, 3


def _layers():
    torch.manual_seed(0)
    return [nn.Sequential(nn.Linear(H, H), nn.Tanh()) for _ in range(L)] + [nn.Linear(H, 4)]


def _data(seed=3):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(MB, H, generator=g), torch.randint(0, 4, (MB, ), generator=g)) for _ in range(STEPS * M)]


def _ref():
    model = nn.Sequential(*_layers())
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    data = _data()
    losses = []
    for s in range(STEPS):
        opt.zero_grad()
        tot = 0.0
        for m in range(M):
            x, y = data[s * M + m]
            loss = nn.functional.cross_entropy(model(x), y) / M
            loss.backward()
            tot += float(loss)
        opt.step()
        losses.append(tot)
    return losses


def _pipe_run(stages, partition, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.pipe import PipelineModule
    net = PipelineModule(layers=_layers(), num_stages=stages, loss_fn=nn.functional.cross_entropy,
                         partition_method=partition)
    cfg = {"train_micro_batch_size_per_gpu": MB, "gradient_accumulation_steps": M,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}}, "steps_per_print": 1000}
    eng, _, _, _ = ds.initialize(model=net, config=cfg)
    it = iter(_data())
    losses = [float(eng.train_batch(it)) for _ in range(STEPS)]
    if dist.get_rank() == 0:
        torch.save(losses, out)


@pytest.mark.parametrize("stages,partition", [(2, "parameters"), (2, "uniform"), (4, "type:sequential")])
def test_pipe_matches_sequential(stages, partition, tmp_path):
    out = str(tmp_path / "l.pt")
    run_distributed(_pipe_run, stages, stages, partition, out)
    got = torch.load(out)
    assert got == pytest.approx(_ref(), rel=1e-4, abs=1e-5)


def test_schedule_1f1b_counts():
    from deepspeedsyclsupport_amd.runtime.pipe import schedule as S
    for stages in (1, 2, 4):
        for sid in range(stages):
            cmds = [c for step in S.TrainSchedule(8, stages, sid) for c in step]
            assert sum(isinstance(c, S.ForwardPass) for c in cmds) == 8
            assert sum(isinstance(c, S.BackwardPass) for c in cmds) == 8
            assert isinstance(cmds[-1], S.OptimizerStep)
            # 1F1B: in-flight micro-batches never exceed the buffer count
            inflight = peak = 0
            for c in cmds:
                inflight += isinstance(c, S.ForwardPass) - isinstance(c, S.BackwardPass)
                peak = max(peak, inflight)
            assert peak <= S.TrainSchedule(8, stages, sid).num_pipe_buffers()


def test_partition_balanced():
    from deepspeedsyclsupport_amd.runtime.pipe.module import partition_balanced, partition_uniform
    assert partition_uniform(10, 2) == [0, 5, 10]
    p = partition_balanced([1, 1, 1, 10, 1, 1], 2)
    assert p[0] == 0 and p[-1] == 6 and len(p) == 3


def test_topology_radix_math():
    """Mixed-radix topology (reference semantics of `runtime/pipe/topology.py`): coordinates, axis communicators,
    filters and rank strings agree with a brute-force enumeration."""
    import itertools
    from deepspeedsyclsupport_amd.runtime.pipe.topology import ProcessTopology, PipeModelDataParallelTopology
    topo = PipeModelDataParallelTopology(num_pp=2, num_mp=2, num_dp=3)
    axes, dims = topo.get_axis_names(), [2, 3, 2]
    brute = {c: r for r, c in enumerate(itertools.product(*[range(d) for d in dims]))}
    for c, r in brute.items():
        assert topo.get_rank(**dict(zip(axes, c))) == r
        assert tuple(topo.get_coord(r)) == c
    for axis in axes:
        k = axes.index(axis)
        lists = topo.get_axis_comm_lists(axis)
        assert sorted(sum(lists, [])) == list(range(12))
        for l in lists:
            cs = [topo.get_coord(r) for r in l]
            assert [c[k] for c in cs] == list(range(dims[k]))
            assert len({tuple(v for i, v in enumerate(c) if i != k) for c in cs}) == 1
    assert topo.filter_match(pipe=1, model=0) == [r for c, r in brute.items() if c[0] == 1 and c[2] == 0]
    assert topo.get_rank_repr(5) == "model_01"
    assert ProcessTopology(["a"], [4]).get_axis_comm_lists("b") == []


def _tied_specs():
    from deepspeedsyclsupport_amd.pipe import LayerSpec, TiedLayerSpec
    # the same [H, H] matrix is the input projection (x W^T) on the first stage and the transposed output projection
    # (x W) on the last stage: the reference's tied embedding / LM head pattern (`tests/unit/pipe/test_pipe_module.py`)
    return ([TiedLayerSpec("tied", nn.Linear, H, H, bias=False)] +
            [LayerSpec(nn.Sequential, nn.Linear(H, H), nn.Tanh()) for _ in range(4)] +
            [TiedLayerSpec("tied", nn.Linear, H, H, bias=False, forward_fn=lambda m, x: x @ m.weight),
             LayerSpec(nn.Linear, H, 4)])


def _tied_run(stages, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.pipe import PipelineModule
    net = PipelineModule(layers=_tied_specs(), num_stages=stages, loss_fn=nn.functional.cross_entropy,
                         partition_method="uniform", seed_layers=True)
    cfg = {"train_micro_batch_size_per_gpu": MB, "gradient_accumulation_steps": M,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}}, "steps_per_print": 1000}
    eng, _, _, _ = ds.initialize(model=net, config=cfg)
    it = iter(_data())
    losses = [float(eng.train_batch(it)) for _ in range(STEPS)]
    tied = [w.detach().clone() for w, _ in net.get_tied_weights_and_groups()] if hasattr(
        net, "get_tied_weights_and_groups") else []
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, [t.sum().item() for t in tied])
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "tied": gathered}, out)


def test_pipe_tied_layers_match_single_stage(tmp_path):
    """TiedLayerSpec across the first and last stage: copies start equal (broadcast), their gradients are
    all-reduced over the tie group every step, so 2 stages train exactly like 1 stage holding one shared module."""
    res = {}
    for stages in (1, 2):
        out = str(tmp_path / f"t{stages}.pt")
        run_distributed(_tied_run, stages, stages, out)
        res[stages] = torch.load(out)
    assert res[2]["losses"] == pytest.approx(res[1]["losses"], rel=1e-4, abs=1e-5)
    t = res[2]["tied"]
    assert len(t) == 2 and t[0] and t[0] == pytest.approx(t[1], rel=1e-6)
