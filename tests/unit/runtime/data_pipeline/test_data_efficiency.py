"""Data efficiency (reference `tests/unit/runtime/test_data_efficiency.py`, curriculum scheduler tests)."""
import numpy as np
import pytest
import torch

from deepspeedsyclsupport_amd.runtime.data_pipeline import CurriculumScheduler
from deepspeedsyclsupport_amd.runtime.data_pipeline.data_routing import RandomLayerTokenDrop, RandomLTDScheduler
from deepspeedsyclsupport_amd.runtime.data_pipeline.data_sampling import DeepSpeedDataSampler


def test_fixed_linear_and_root():
    c = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_linear",
                             "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 8}})
    seq = [c.update_difficulty(s) for s in range(0, 14)]
    assert seq[0] == 8 and seq[-1] == 64 and all(b >= a for a, b in zip(seq, seq[1:]))
    assert all(v % 8 == 0 for v in seq)
    r = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_root",
                             "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 8,
                                                 "root_degree": 2}})
    assert r.get_difficulty(2) >= c.get_difficulty(2)  # root schedules ramp faster early


def test_fixed_discrete_and_custom():
    c = CurriculumScheduler({"min_difficulty": 1, "max_difficulty": 3, "schedule_type": "fixed_discrete",
                             "schedule_config": {"difficulty": [1, 2, 3], "max_step": [5, 10]}})
    assert [c.get_difficulty(s) for s in (0, 5, 6, 10, 11, 100)] == [1, 1, 2, 2, 3, 3]
    cu = CurriculumScheduler({"min_difficulty": 0, "max_difficulty": 10, "schedule_type": "custom"})
    cu.set_custom_get_difficulty(lambda s: min(s, 10))
    assert cu.update_difficulty(4) == 4
    with pytest.raises(AssertionError):
        CurriculumScheduler({"min_difficulty": 1, "max_difficulty": 3, "schedule_type": "fixed_discrete",
                             "schedule_config": {"difficulty": [1, 2], "max_step": [5, 10]}})


def test_curriculum_sampler_respects_difficulty():
    vals = np.arange(100)  # difficulty = sample index
    cfg = {"seed": 3, "data_sampling": {"curriculum_learning": {"curriculum_metrics": {"seqlen": {
        "min_difficulty": 10, "max_difficulty": 100, "schedule_type": "fixed_linear",
        "schedule_config": {"total_curriculum_step": 5, "difficulty_step": 10}}}}}}
    s0 = DeepSpeedDataSampler(cfg, 100, 2, 0, 2, metric_values={"seqlen": vals})
    first = s0.get_next_global_batch()
    assert first.max() <= 20
    later = [s0.get_next_global_batch() for _ in range(6)][-1]
    assert later.max() > 20
    # ranks see disjoint slices of the same global batch
    a = DeepSpeedDataSampler(cfg, 16, 2, 0, 2, metric_values={"seqlen": vals[:16]})
    b = DeepSpeedDataSampler(cfg, 16, 2, 1, 2, metric_values={"seqlen": vals[:16]})
    ia, ib = next(iter(a)), next(iter(b))
    assert len(ia) == 2 and len(ib) == 2 and not set(ia) & set(ib)


def test_random_ltd_layer():
    torch.manual_seed(0)
    lin = torch.nn.Linear(8, 8)
    layer = RandomLayerTokenDrop(lin)
    sch = RandomLTDScheduler({"random_ltd_schedule": {"min_value": 4, "max_value": 16,
                                                      "schedule_config": {"require_steps": 4, "seq_per_step": 4}}})
    layer.init_config({}, sch, 0)
    x = torch.randn(2, 16, 8)
    y = layer(x)
    changed = (y != x).any(-1)
    assert changed.sum(1).tolist() == [4, 4]  # exactly the kept tokens went through the layer
    sch.update_seq(4)
    assert sch.get_current_seq() == 16
    torch.testing.assert_close(layer(x), lin(x))
    layer.eval()
    sch.set_current_seq(4)
    torch.testing.assert_close(layer(x), lin(x))


def test_random_ltd_mask_slicing():
    """Encoder masks are gathered on both axes at the kept positions, decoder causal masks keep their k x k corner
    (reference `ops/random_ltd/dropping_utils.py` bert/gpt_sample_tokens)."""
    from deepspeedsyclsupport_amd.runtime.data_pipeline.data_routing.basic_layer import (RandomLayerTokenDrop,
                                                                                          mask_gather_bert,
                                                                                          mask_gather_gpt)
    B, S, k = 2, 6, 3
    full = torch.arange(B * S * S, dtype=torch.float32).view(B, 1, S, S)
    idx = torch.tensor([[0, 2, 5], [1, 3, 4]])
    got = mask_gather_bert(full, idx)
    for b in range(B):
        torch.testing.assert_close(got[b, 0], full[b, 0][idx[b]][:, idx[b]])
    pad = torch.arange(B * S, dtype=torch.float32).view(B, 1, 1, S)
    torch.testing.assert_close(mask_gather_bert(pad, idx)[:, 0, 0], torch.gather(pad[:, 0, 0], 1, idx))
    causal = torch.tril(torch.ones(S, S)).view(1, 1, S, S)
    torch.testing.assert_close(mask_gather_gpt(causal, k), torch.tril(torch.ones(k, k)).view(1, 1, k, k))

    class Layer(torch.nn.Module):

        def forward(self, x, attention_mask=None):
            self.seen = attention_mask.shape
            return x * 2

    class Sched:

        def get_current_seq(self):
            return k

    lyr = RandomLayerTokenDrop(Layer())
    lyr.init_config({"model_mask_name": "attention_mask", "model_type": "encoder"}, Sched(), 0)
    lyr.train()
    x = torch.randn(B, S, 4)
    out = lyr(x, attention_mask=full)
    assert lyr.random_ltd_layer.seen == (B, 1, k, k)
    changed = (out != x).any(-1).sum(1)
    assert changed.tolist() == [k, k]


def test_random_ltd_ops_frontend():
    """ops/random_ltd: sampled indices are sorted and distinct; GatherTokens / ScatterTokens are exact adjoints."""
    from deepspeedsyclsupport_amd.ops.random_ltd import GatherTokens, ScatterTokens, gpt_sample_tokens
    idx, mask = gpt_sample_tokens(4, 10, 3, layers=2, attn_mask=torch.tril(torch.ones(1, 1, 10, 10)))
    assert idx.shape == (2, 3, 4) and idx.dtype == torch.int32 and mask.shape == (1, 1, 4, 4)
    assert (idx[..., 1:] > idx[..., :-1]).all()
    x = torch.randn(3, 10, 8, requires_grad=True)
    acts, part = GatherTokens.apply(x, idx[0], True)
    torch.testing.assert_close(part, torch.stack([x[b, idx[0, b].long()] for b in range(3)]))
    full = ScatterTokens.apply(acts, part * 2, idx[0], True)
    full.sum().backward()
    # kept tokens were doubled and scattered back over themselves: d/dx = 2 on the kept set, 1 (bypass) elsewhere
    g = x.grad
    for b in range(3):
        keep = set(idx[0, b].tolist())
        for s in range(10):
            assert torch.allclose(g[b, s], torch.full((8, ), 2.0 if s in keep else 1.0))


def test_utils_reference_paths():
    from deepspeedsyclsupport_amd.utils import debug, numa
    from deepspeedsyclsupport_amd.utils.groups import _get_data_parallel_world_size  # noqa: F401
    from deepspeedsyclsupport_amd.utils.types import GATED_ACTIVATION_TYPES, ActivationFuncType
    assert ActivationFuncType.GATED_SILU in GATED_ACTIVATION_TYPES
    assert numa.parse_range_list("0-2,5,7-8") == [0, 1, 2, 5, 7, 8]
    per, cmd = numa.get_numactl_cmd("0-7", 4, 2)
    assert per == 2 and cmd[0] == "numactl" and cmd[-1] == "4,5"
    m = torch.nn.Linear(2, 2)
    debug.debug_extract_module_and_param_names(m)
    assert debug.debug_param2name(m.weight) == "weight"
