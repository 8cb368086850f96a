"""MoE checkpoints (reference `tests/unit/checkpoint/test_moe_checkpoint.py`, engine `_save_moe_checkpoint` /
`load_moe_state_dict`, `runtime/engine.py:2534-2600, 3151-3258`): world 4 with expert-parallel size 2 (so every
expert is replicated on 2 expert-data-parallel ranks and partitioned over them by ZeRO-2).

* one `layer_{l}_expert_{e}_mp_rank_00_model_states.pt` per GLOBAL expert id, written by expert-DP rank 0;
* zero_to_fp32 reassembles expert parameters under their global ids from the ranks' own layouts (expert-parallel
  ranks hold different experts under the same local names, so a rank-0-structure reassembly would overwrite them);
* reload at world 4 (positional) and at world 2 (re-partitioned) restores every fp32 master and moment.
"""
import os

import pytest
import torch
import torch.nn as nn

from ..common import run_distributed

H, E = 16, 4


class MoEModel(nn.Module):

    def __init__(self, seed=0):
        super().__init__()
        from deepspeedsyclsupport_amd.moe import MoE
        torch.manual_seed(seed)
        self.inp = nn.Linear(H, H)
        expert = nn.Sequential(nn.Linear(H, 2 * H), nn.GELU(), nn.Linear(2 * H, H))
        self.moe = MoE(H, expert, num_experts=E, ep_size=2, k=1, drop_tokens=False, use_rts=False)
        self.out = nn.Linear(H, 4)

    def forward(self, x, y):
        h, _, _ = self.moe(torch.relu(self.inp(x)))
        return nn.functional.cross_entropy(self.out(h), y)


def _cfg():
    return {"train_micro_batch_size_per_gpu": 6, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
            "zero_optimization": {"stage": 2, "reduce_bucket_size": 500}, "gradient_clipping": 0.0}


def _state(eng):
    from deepspeedsyclsupport_amd.checkpoint.zero_checkpoint import global_param_names
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    g = global_param_names(eng.module)
    return {g[n]: (safe_get_full_fp32_param(p), safe_get_full_optimizer_state(p, "exp_avg"))
            for n, p in eng.module.named_parameters()}


def _save(ckpt, outdir):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    rank = dist.get_rank()
    eng, _, _, _ = ds.initialize(model=MoEModel(seed=rank // 2), config=_cfg())  # EP ranks differ in experts
    gen = torch.Generator().manual_seed(rank)
    x, y = torch.randn(6, H, generator=gen), torch.randint(0, 4, (6, ), generator=gen)
    loss = eng(x, y)
    eng.backward(loss)
    eng.step()
    eng.save_checkpoint(ckpt, tag="m")
    torch.save(_state(eng), os.path.join(outdir, f"state{rank}.pt"))


def _load(ckpt, outdir):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    eng, _, _, _ = ds.initialize(model=MoEModel(seed=77), config=_cfg())
    eng.load_checkpoint(ckpt, tag="m")
    ref = {}
    for f in os.listdir(outdir):
        if f.startswith("state"):
            ref.update(torch.load(os.path.join(outdir, f), weights_only=True))
    for name, (w, m) in _state(eng).items():
        torch.testing.assert_close(w, ref[name][0], rtol=0, atol=0, msg=name)
        torch.testing.assert_close(m, ref[name][1], rtol=0, atol=0, msg=name)
    assert dist.get_world_size() in (2, 4)


def test_moe_checkpoint_expert_files_consolidation_and_reload(tmp_path):
    ckpt, outdir = str(tmp_path / "ck"), str(tmp_path / "st")
    os.makedirs(outdir)
    run_distributed(_save, 4, ckpt, outdir)
    files = os.listdir(os.path.join(ckpt, "m"))
    for e in range(E):
        assert f"layer_0_expert_{e}_mp_rank_00_model_states.pt" in files, files
    ref = {}
    for f in os.listdir(outdir):
        ref.update(torch.load(os.path.join(outdir, f), weights_only=True))
    # the two expert-parallel ranks trained different experts (different seeds): all 4 global experts present
    assert any("deepspeed_experts.3." in k for k in ref)
    from deepspeedsyclsupport_amd.utils.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
    sd = get_fp32_state_dict_from_zero_checkpoint(ckpt, tag="m")
    for name, (w, _) in ref.items():
        torch.testing.assert_close(sd[name], w, rtol=0, atol=0, msg=name)
    # expert file contents match the 16-bit expert weights under global ids
    e3 = torch.load(os.path.join(ckpt, "m", "layer_0_expert_3_mp_rank_00_model_states.pt"), weights_only=True)
    for k, v in e3.items():
        assert "deepspeed_experts.3." in k
        torch.testing.assert_close(v.float(), ref[k][0], rtol=0, atol=0)
    run_distributed(_load, 4, ckpt, outdir)
    run_distributed(_load, 2, ckpt, outdir)
