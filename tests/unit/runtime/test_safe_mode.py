"""ZeRO `safe_mode` cross-rank consistency checks (reference `runtime/zero/utils.py:60-89`
`assert_ints_same_as_other_ranks`, all-gather / reduce `safe_mode`, coordinator trace validation): a healthy run is
unaffected; ranks that diverge (different module order -> different collective order) raise on EVERY rank instead
of deadlocking or silently mixing buffers."""
import pytest
import torch
import torch.nn as nn

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama


def _healthy(stage):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    cfg = base_config(stage=stage)
    cfg["zero_optimization"]["safe_mode"] = True
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    for x in random_tokens(3, 2, 16, seed=dist.get_rank()):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
    assert torch.isfinite(loss)


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_safe_mode_healthy_run(stage):
    run_distributed(_healthy, 2, stage)


class Branchy(nn.Module):

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = nn.Linear(64, 64)
        self.b = nn.Linear(64, 64)
        self.head = nn.Linear(64, 1)

    def forward(self, x, order):
        for m in ([self.a, self.b] if order == 0 else [self.b, self.a]):
            x = torch.relu(m(x))
        return self.head(x).pow(2).mean()


def _divergent():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.zero.utils import ZeRORuntimeException
    cfg = base_config(stage=3)
    cfg["zero_optimization"].update(safe_mode=True, stage3_param_persistence_threshold=0)
    eng, _, _, _ = ds.initialize(model=Branchy(), config=cfg)
    x = torch.randn(4, 64)
    with pytest.raises(ZeRORuntimeException, match="differ across ranks"):
        loss = eng(x, dist.get_rank())  # rank 0 runs a then b, rank 1 b then a
        eng.backward(loss)
        eng.step()


def test_safe_mode_detects_divergent_collective_order():
    run_distributed(_divergent, 2)


def test_assert_ints_same_single_process_is_noop():
    from deepspeedsyclsupport_amd.runtime.zero.utils import assert_ints_same_as_other_ranks, trace_digest
    assert_ints_same_as_other_ranks([1, 2, 3])
    assert trace_digest([1, 2, 3]) != trace_digest([1, 3, 2])
