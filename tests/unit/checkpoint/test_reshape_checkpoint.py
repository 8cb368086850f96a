"""3-D checkpoint folder inspection and contraction (reference `tests/unit/checkpoint/test_reshape_checkpoint.py`:
2-D / 3-D maps for (pp, tp, dp) contractions) on a synthetic Megatron-DeepSpeed style folder."""
import os

import pytest
import torch

from deepspeedsyclsupport_amd.checkpoint import constants as CK
from deepspeedsyclsupport_amd.checkpoint.deepspeed_checkpoint import DeepSpeedCheckpoint, ZeROCheckpoint
from deepspeedsyclsupport_amd.checkpoint.reshape_3d_utils import get_model_3d_descriptor, model_3d_desc
from deepspeedsyclsupport_amd.checkpoint.reshape_meg_2d import get_mpu_ranks, reshape_meg_2d_parallel
from deepspeedsyclsupport_amd.checkpoint.utils import (clone_tensors_for_torch_save, get_layer_ckpt_name_for_rank,
                                                       get_model_ckpt_name_for_rank, get_zero_ckpt_name_for_rank)


def test_2d_contraction_maps():
    m = reshape_meg_2d_parallel(old_pp_degree=2, old_tp_degree=4, new_pp_degree=2, new_tp_degree=2)
    assert [m.get_data(0, 0), m.get_data(0, 1), m.get_data(1, 0), m.get_data(1, 1)] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    m = reshape_meg_2d_parallel(2, 4, 1, 4)  # pipeline stages merge per tensor-parallel column
    assert [m.get_data(0, j) for j in range(4)] == [[0, 4], [1, 5], [2, 6], [3, 7]]
    m = reshape_meg_2d_parallel(2, 2, 1, 1)
    assert m.get_data(0, 0) == [0, 1, 2, 3]
    with pytest.raises(ValueError):
        reshape_meg_2d_parallel(1, 2, 2, 2)


def test_3d_contraction_maps():
    src = model_3d_desc(pp_degree=2, tp_degree=2, dp_degree=2)
    ok, errs = src.can_reshape(model_3d_desc(2, 2, 4))
    assert not ok and "DP" in errs[0]
    maps = src.reshape(model_3d_desc(pp_degree=1, tp_degree=2, dp_degree=1))
    assert len(maps) == 1
    # file index = model rank + dp_index * 4; cell (0, tp) merges both pipeline stages and both dp ranks
    assert maps[0].get_data(0, 0) == [0, 4, 2, 6] and maps[0].get_data(0, 1) == [1, 5, 3, 7]
    same = src.reshape(model_3d_desc(2, 2, 2))
    assert [same[d].get_data(p, t) for d in range(2) for p in range(2) for t in range(2)] == \
        [[0], [1], [2], [3], [4], [5], [6], [7]]
    assert src.world_size() == 8 and src.is_valid(1, 1, 1)[0] and not src.is_valid(2, 0, 0)[0]


def test_mpu_rank_groups():
    tp, rep, dp = get_mpu_ranks(tp_size=2, pp_size=4, dp_size=2)
    assert tp[:3] == [[0, 1], [2, 3], [4, 5]] and dp[:4] == [[0, 2], [1, 3], [4, 6], [5, 7]]
    assert rep[0] == [0, 1, 4, 5, 8, 9, 12, 13] and len(rep) == 2


def _make_folder(d, pp=2, tp=2, dp=2, layers=4, H=8):
    os.makedirs(d, exist_ok=True)
    torch.manual_seed(0)
    full = {}
    for mp in range(pp * tp):
        torch.save({"iteration": 7, "args": {"hidden": H}, "module": {}, "checkpoint_info": {"k": 1}},
                   get_model_ckpt_name_for_rank(d, f"{mp:02d}"))
    keys = ["layer_00"] + [f"layer_{i + 1:02d}" for i in range(layers)] + [f"layer_{layers + 1:02d}"]
    for key in keys:
        if key == keys[0]:
            sd_full = {"word_embeddings.weight": torch.randn(16, H), "position_embeddings.weight": torch.randn(4, H)}
        elif key == keys[-1]:
            sd_full = {"weight": torch.randn(H), "bias": torch.randn(H)}
        else:
            sd_full = {"input_layernorm.weight": torch.randn(H), "self_attention.query_key_value.weight":
                       torch.randn(3 * H, H), "self_attention.dense.weight": torch.randn(H, H),
                       "mlp.dense_4h_to_h.bias": torch.randn(H)}
        full[key] = sd_full
        for t in range(tp):
            part = {}
            for k, v in sd_full.items():
                if k in ("input_layernorm.weight", "mlp.dense_4h_to_h.bias", "position_embeddings.weight") or \
                        key == keys[-1]:
                    part[k] = v.clone()
                elif k == "self_attention.dense.weight":
                    part[k] = v.chunk(tp, 1)[t].clone()
                else:
                    part[k] = v.chunk(tp, 0)[t].clone()
            torch.save(part, get_layer_ckpt_name_for_rank(d, key, t))
    for r in range(dp):
        for mp in range(pp * tp):
            n = 10
            osd = {CK.ZERO_STAGE: 1, CK.PARTITION_COUNT: [dp], CK.GROUP_PADDINGS: [2 if r == dp - 1 else 0],
                   CK.BASE_OPTIMIZER_STATE: {"state": {0: {"exp_avg": torch.full((n, ), float(r * 100 + mp)),
                                                           "step": 3}},
                                             "param_groups": [{"params": [0]}]},
                   CK.SINGLE_PARTITION_OF_FP32_GROUPS: [torch.full((n - (2 if r == dp - 1 else 0), ),
                                                                   float(r * 100 + mp))]}
            torch.save({CK.OPTIMIZER_STATE_DICT: osd}, get_zero_ckpt_name_for_rank(d, r, mp))
    return full, keys


def test_deepspeed_checkpoint_inspects_and_merges(tmp_path):
    d = str(tmp_path / "global_step7")
    full, keys = _make_folder(d)
    desc = get_model_3d_descriptor(d)
    assert (desc.pp_degree, desc.tp_degree, desc.dp_degree) == (2, 2, 2)
    ck = DeepSpeedCheckpoint(d)
    assert (ck.tp_degree, ck.pp_degree, ck.dp_degree) == (2, 2, 2) and ck.original_world_size == 8
    assert ck.get_iteration() == 7 and ck.get_args() == {"hidden": 8} and ck.get_checkpoint_info() == {"k": 1}
    assert ck.layer_keys == keys and ck.get_embedding_layer_id() == "layer_00"
    assert ck.get_pp_transformer_map(0) == keys[1:3] and ck.get_pp_transformer_map(1) == keys[3:5]
    assert len(ck.get_zero_files(1, 1, 1)) == 1 and ck.get_zero_files(1, 1, 1)[0].endswith("rank_1_mp_rank_03_optim_states.pt")
    # contraction to tp=1, pp=1, dp=1: every layer's slices merge back to the full tensors
    one = DeepSpeedCheckpoint(d, tp_degree=1, pp_degree=1, dp_degree=1)
    assert one.is_change_tp_degree() and one.is_change_pp_degree() and one.is_change_dp_degree()
    emb = one.get_embedding_state(0)
    torch.testing.assert_close(emb["word_embeddings.weight"], full["layer_00"]["word_embeddings.weight"])
    torch.testing.assert_close(emb["position_embeddings.weight"], full["layer_00"]["position_embeddings.weight"])
    tstates = one.get_transformer_state(tp_index=0, pp_index=0)
    assert len(tstates) == 4
    for key, sd in zip(keys[1:-1], tstates):
        for k, v in full[key].items():
            torch.testing.assert_close(sd[k], v, msg=f"{key} {k}")
    torch.testing.assert_close(one.get_final_norm_state(0)["weight"], full[keys[-1]]["weight"])
    assert len(one.get_2d_parallel_files(tp_index=0, pp_index=0)) == 4
    # the merged ZeRO state of the single target rank: 8 partitions, paddings stripped, counts rewritten
    z = one.get_zero_checkpoint_state(0, 0, 0)[CK.OPTIMIZER_STATE_DICT]
    assert z[CK.PARTITION_COUNT] == [1] and z[CK.GROUP_PADDINGS] == [0]
    assert z[CK.SINGLE_PARTITION_OF_FP32_GROUPS][0].numel() == 4 * 10 + 4 * 8
    assert z[CK.BASE_OPTIMIZER_STATE]["state"][0]["exp_avg"].numel() == 4 * 10 + 4 * 8
    zc = ZeROCheckpoint(d)
    assert zc.get_src_world_size() == 8 and zc.get_file_indices_for_rank(1, 0, 1) == [6]


def test_clone_tensors_for_torch_save_shrinks_views(tmp_path):
    big = torch.zeros(1 << 16)
    state = {"a": big[:8], "b": [big[8:16], 3], "c": ("x", big[16:24])}
    a, b = str(tmp_path / "raw.pt"), str(tmp_path / "cloned.pt")
    torch.save(state, a)
    cloned = clone_tensors_for_torch_save(state)
    torch.save(cloned, b)
    assert os.path.getsize(b) < os.path.getsize(a) / 10
    assert cloned["b"][1] == 3 and cloned["c"][0] == "x" and torch.equal(cloned["a"], state["a"])
