"""Pipeline checkpoints (reference `tests/unit/checkpoint/test_pipeline.py`): per-layer files indexed by global layer
number; a run resumes exactly under the same topology and its weights load under another stage count."""
import glob
import os

import pytest
import torch
import torch.nn as nn

from ..common import run_distributed

H, L, M, MB = 16, 5, 2, 2


def _layers():
    torch.manual_seed(0)
    return [nn.Sequential(nn.Linear(H, H), nn.Tanh()) for _ in range(L)] + [nn.Linear(H, 4)]


def _data(n, seed=3):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(MB, H, generator=g), torch.randint(0, 4, (MB, ), generator=g)) for _ in range(n * M)]


def _engine(stages, zero_stage=1, parallel_write=False):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.pipe import PipelineModule
    net = PipelineModule(layers=_layers(), num_stages=stages, loss_fn=nn.functional.cross_entropy,
                         partition_method="uniform")
    cfg = {"train_micro_batch_size_per_gpu": MB, "gradient_accumulation_steps": M, "steps_per_print": 1000,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}},
           "zero_optimization": {"stage": zero_stage},
           "checkpoint": {"parallel_write": {"pipeline_stage": parallel_write}}}
    eng, *_ = ds.initialize(model=net, config=cfg)
    return eng


def _resume(stages, save_dir, out, parallel_write):
    from deepspeedsyclsupport_amd import comm as dist
    eng = _engine(stages, parallel_write=parallel_write)
    data = _data(5)
    it = iter(data)
    for _ in range(2):
        eng.train_batch(it)
    eng.save_checkpoint(save_dir, tag="s2")
    cont = [float(eng.train_batch(it)) for _ in range(3)]
    eng2 = _engine(stages, parallel_write=parallel_write)
    eng2.load_checkpoint(save_dir)
    it = iter(data[2 * M:])
    again = [float(eng2.train_batch(it)) for _ in range(3)]
    if dist.get_rank() == 0:
        torch.save({"cont": cont, "again": again, "steps": eng2.global_steps,
                    "files": sorted(os.path.basename(f) for f in glob.glob(os.path.join(save_dir, "s2", "*")))}, out)


@pytest.mark.parametrize("world,stages,parallel_write", [(2, 2, False), (4, 2, True)])
def test_pipeline_checkpoint_resumes(world, stages, parallel_write, tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_resume, world, stages, str(tmp_path / "ck"), out, parallel_write)
    res = torch.load(out)
    assert res["again"] == pytest.approx(res["cont"], rel=1e-6, abs=1e-7)
    files = res["files"]
    # one file per layer (global numbering), one model-states file per stage, one optimizer shard per rank
    assert [f for f in files if f.startswith("layer_")] == [f"layer_{i:02d}-model_states.pt" for i in range(L + 1)]
    assert [f for f in files if f.startswith("mp_rank_")] == [f"mp_rank_{s:02d}_model_states.pt"
                                                             for s in range(stages)]
    assert len([f for f in files if f.endswith("_optim_states.pt")]) == world


def _save_weights(stages, save_dir, out):
    from deepspeedsyclsupport_amd import comm as dist
    eng = _engine(stages, zero_stage=0)
    it = iter(_data(2))
    for _ in range(2):
        eng.train_batch(it)
    eng.save_checkpoint(save_dir, tag="w")
    sd = {k: v.detach().clone() for k, v in eng.module.state_dict().items()}
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, sd)
    if dist.get_rank() == 0:
        torch.save({k: v for d in got for k, v in d.items()}, out)


def _load_weights(stages, save_dir, out):
    from deepspeedsyclsupport_amd import comm as dist
    eng = _engine(stages, zero_stage=0)
    eng.load_checkpoint(save_dir, load_module_only=True)
    sd = {k: v.detach().clone() for k, v in eng.module.state_dict().items()}
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, sd)
    # the fp32 masters follow the loaded weights: one more step moves away from them, not from the initial ones
    if dist.get_rank() == 0:
        torch.save({k: v for d in got for k, v in d.items()}, out)


@pytest.mark.parametrize("save_stages,load_stages", [(2, 1), (1, 2), (2, 3)])
def test_pipeline_checkpoint_loads_under_another_stage_count(save_stages, load_stages, tmp_path):
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    run_distributed(_save_weights, save_stages, save_stages, str(tmp_path / "ck"), a)
    run_distributed(_load_weights, load_stages, load_stages, str(tmp_path / "ck"), b)
    saved, loaded = torch.load(a), torch.load(b)
    assert saved.keys() == loaded.keys() and len(saved) == 2 * (L + 1)
    for k in saved:
        assert torch.equal(saved[k], loaded[k]), k
    # and it is not the initial state
    init = nn.Sequential(*_layers()).state_dict()
    assert any(not torch.equal(init[k], saved[k]) for k in saved)
