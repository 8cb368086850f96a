"""Inspecting and re-shaping 3-D parallel checkpoint folders (reference `checkpoint/deepspeed_checkpoint.py:33-290`
`DeepSpeedCheckpoint`, `checkpoint/zero_checkpoint.py:17-140` `ZeROCheckpoint`).

A Megatron-DeepSpeed checkpoint folder holds `mp_rank_XX_model_states.pt` per model-parallel rank, optionally
`layer_NN-model_TT-model_states.pt` per pipeline layer and tensor-parallel rank, and one ZeRO optimizer file per
(data, model)-parallel rank. Both classes answer "which source files does target rank (pp, tp, dp) read" for a
target topology that is the source's or a contraction of it, and merge the states of those files: tensor-parallel
slices concatenate (row-parallel weights on dim 1, replicated layers taken once), ZeRO partitions concatenate with
their alignment padding stripped.

Files are read with `weights_only=True` (`zero_checkpoint.load_file`): nothing in them is executed.
"""
import os

import torch

from . import constants as CK
from .reshape_3d_utils import get_model_3d_descriptor, model_3d_desc
from .reshape_meg_2d import meg_2d_parallel_map, reshape_meg_2d_parallel
from .reshape_utils import (basic_folder_validation, get_files, get_files_with_prefix, get_zero_files, merge_state,
                            partition_data)
from .zero_checkpoint import load_file

EMBEDDING_LAYER_INDEX = 0
FINAL_LAYER_NORM_INDEX = -1
ARGS_KEY = "args"
CHECKPOINT_INFO_KEY = "checkpoint_info"
ITERATION_KEY = "iteration"
GROUP_STATE_KEY = "state"
# tensor-parallel merge rules of Megatron's transformer layer: replicated entries, and the concat dim of the rest
SEQUENTIAL_LAYERS = ("input_layernorm.weight", "input_layernorm.bias", "self_attention.dense.bias",
                     "post_attention_layernorm.weight", "post_attention_layernorm.bias", "mlp.dense_4h_to_h.bias",
                     "position_embeddings.weight")
LAYER_CONCAT_DIM = {"self_attention.dense.weight": 1, "mlp.dense_4h_to_h.weight": 1}


class ZeROCheckpoint:
    """The ZeRO optimizer files of a folder as a (pp, tp, dp) grid, re-mappable onto a smaller grid."""

    def __init__(self, dir):
        basic_folder_validation(dir)
        self.dir = dir
        self.file_list = get_zero_files(dir)
        self.num_files = len(self.file_list)
        if not self.num_files:
            raise FileNotFoundError(f"No ZeRO files found in {dir}")
        self.src_3d = get_model_3d_descriptor(dir)
        self.reshape(model_3d_desc(self.src_3d.pp_degree, self.src_3d.tp_degree, self.src_3d.dp_degree))

    def reshape(self, target_3d_desc):
        self.target_3d = target_3d_desc
        self._3d_file_map = self.src_3d.reshape(target_3d_desc)

    def get_src_world_size(self):
        return self.src_3d.world_size()

    def get_src_tp_degree(self):
        return self.src_3d.tp_degree

    def get_src_pp_degree(self):
        return self.src_3d.pp_degree

    def get_src_dp_degree(self):
        return self.src_3d.dp_degree

    def get_file_indices_for_rank(self, pp_index, tp_index, dp_index):
        if dp_index >= len(self._3d_file_map):
            raise IndexError(f"DP index {dp_index} >= DP degree {len(self._3d_file_map)}")
        return self._3d_file_map[dp_index].get_data(pp_index, tp_index)

    def get_files_for_rank(self, pp_index, tp_index, dp_index):
        return [self.file_list[i] for i in self.get_file_indices_for_rank(pp_index, tp_index, dp_index)]

    def get_state_for_rank(self, pp_index, tp_index, dp_index, keys_to_ignore=(), strip_tensor_paddings=True):
        """Merged optimizer state of the source files target rank (pp, tp, dp) covers."""
        merged = None
        for f in self.get_files_for_rank(pp_index, tp_index, dp_index):
            sd = load_file(f, mmap=False)
            for k in keys_to_ignore:
                sd.pop(k, None)
            if strip_tensor_paddings:
                self._strip_tensor_paddings(sd)
            merged = sd if merged is None else merge_state(merged, sd)
            osd = merged.get(CK.OPTIMIZER_STATE_DICT) or {}
            if osd.get(CK.PARTITION_COUNT):
                osd[CK.PARTITION_COUNT] = [self.target_3d.dp_degree] * len(osd[CK.PARTITION_COUNT])
            if strip_tensor_paddings and osd.get(CK.GROUP_PADDINGS):
                osd[CK.GROUP_PADDINGS] = [0] * len(osd[CK.GROUP_PADDINGS])
        return merged

    @staticmethod
    def _strip_tensor_paddings(sd):
        osd = sd.get(CK.OPTIMIZER_STATE_DICT) or {}
        paddings = osd.get(CK.GROUP_PADDINGS)
        states = (osd.get(CK.BASE_OPTIMIZER_STATE) or {}).get(GROUP_STATE_KEY) \
            if isinstance(osd.get(CK.BASE_OPTIMIZER_STATE), dict) else None
        if not paddings or states is None:
            return
        for gi, st in states.items():
            pad = paddings[gi]
            if not pad:
                continue
            for name, v in st.items():
                if torch.is_tensor(v) and v.dim() > 0:
                    st[name] = v.narrow(0, 0, v.numel() - pad).clone()

    def print_3d_index_map(self, tag=None):
        if tag:
            print(f"3D index map: {tag}")
        for d, m in enumerate(self._3d_file_map):
            m.print_data(f"dp = {d}")

    def print_3d_file_map(self, tag=None):
        if tag:
            print(f"3D file map: {tag}")
        for d, m in enumerate(self._3d_file_map):
            for p in range(m.pp_degree):
                for t in range(m.tp_degree):
                    print(f"{p}, {t}, {d} => {[self.file_list[i] for i in m.get_data(p, t)]}")


class DeepSpeedCheckpoint:
    """A checkpoint folder viewed at a target (tp, pp, dp) topology (defaults: the saved one)."""

    def __init__(self, dir, tp_degree=None, pp_degree=None, dp_degree=None):
        self.dir = dir
        basic_folder_validation(dir)
        self.file_list = get_files(dir)
        self.layer_files = [f for f in get_files_with_prefix(self.file_list, CK.LAYER_FILE_PREFIX)
                            if "expert_" not in os.path.basename(f)]
        self.mp_rank_files = [f for f in get_files_with_prefix(self.file_list, CK.MODEL_FILE_PREFIX)
                              if f.endswith(CK.MODEL_FILE_SUFFIX)]
        if not self.mp_rank_files:
            raise FileNotFoundError(f"{dir} seems a bogus DeepSpeed checkpoint folder: Cannot find "
                                    f"{CK.MODEL_FILE_PREFIX}* files in there.")
        self.zero_checkpoint = ZeROCheckpoint(dir)
        src = self.zero_checkpoint.src_3d
        self.layer_keys = sorted({os.path.basename(f)[:len(CK.LAYER_FILE_PREFIX) + 2] for f in self.layer_files})
        self.layer_count = len(self.layer_keys)
        self.tp_degree = src.tp_degree if tp_degree is None else tp_degree
        self.pp_degree = src.pp_degree if pp_degree is None else pp_degree
        self.dp_degree = src.dp_degree if dp_degree is None else dp_degree
        self.original_world_size = src.world_size()
        self.world_size = self.tp_degree * self.pp_degree * self.dp_degree
        self.old_2d_map = meg_2d_parallel_map(src.pp_degree, src.tp_degree)
        self.old_2d_map.simple_init()
        self.new_2d_map = reshape_meg_2d_parallel(src.pp_degree, src.tp_degree, self.pp_degree, self.tp_degree)
        if self.is_change_pp_degree() or self.is_change_tp_degree() or self.is_change_dp_degree():
            self.zero_checkpoint.reshape(model_3d_desc(self.pp_degree, self.tp_degree, self.dp_degree))
        if len(self.mp_rank_files) % self.tp_degree or self.zero_checkpoint.num_files % (self.pp_degree * self.tp_degree):
            raise ValueError(f"{dir}: file counts do not divide the target topology")
        self.global_state = {}
        self.pp_to_transformer_map = self._build_pp_transformer_map()
        self.transformer_file_map = self._build_transformer_file_map()
        self.tp_to_embedding_map = self._build_tp_other_layer_map(EMBEDDING_LAYER_INDEX)
        self.tp_to_final_norm_map = self._build_tp_other_layer_map(FINAL_LAYER_NORM_INDEX)

    # ----------------------------------------------------------------------------------------------- topology
    def is_change_tp_degree(self):
        return self.tp_degree != self.zero_checkpoint.get_src_tp_degree()

    def is_change_pp_degree(self):
        return self.pp_degree != self.zero_checkpoint.get_src_pp_degree()

    def is_change_dp_degree(self):
        return self.dp_degree != self.zero_checkpoint.get_src_dp_degree()

    def get_2d_parallel_files(self, tp_index, pp_index):
        return [self.mp_rank_files[i] for i in self.new_2d_map.get_data(pp_index=pp_index, tp_index=tp_index)]

    def get_zero_files(self, pp_index, tp_index, dp_index):
        return self.zero_checkpoint.get_files_for_rank(pp_index, tp_index, dp_index)

    def get_zero_checkpoint_state(self, pp_index, tp_index, dp_index):
        return self.zero_checkpoint.get_state_for_rank(pp_index, tp_index, dp_index, keys_to_ignore=[CK.PARAM_SHAPES])

    # ----------------------------------------------------------------------------------------------- global values
    def _value(self, key, default=None):
        if key not in self.global_state:
            self.global_state[key] = load_file(self.mp_rank_files[0], mmap=False).get(key, default)
        return self.global_state[key]

    def get_iteration(self):
        return self._value(ITERATION_KEY, 0)

    def get_args(self):
        return self._value(ARGS_KEY)

    def get_checkpoint_info(self, info_key=CHECKPOINT_INFO_KEY):
        return self._value(info_key)

    # ----------------------------------------------------------------------------------------------- layer states
    def get_embedding_layer_id(self):
        return self.layer_keys[EMBEDDING_LAYER_INDEX]

    def get_final_norm_layer_id(self):
        return self.layer_keys[FINAL_LAYER_NORM_INDEX]

    def get_embedding_files(self, tp_index):
        return self.tp_to_embedding_map[tp_index]

    def get_final_norm_files(self, tp_index):
        return self.tp_to_final_norm_map[tp_index]

    def get_embedding_state(self, tp_index):
        return self._merge_state_dicts([load_file(f, mmap=False) for f in self.tp_to_embedding_map[tp_index]])

    def get_final_norm_state(self, tp_index):
        return load_file(self.tp_to_final_norm_map[tp_index][0], mmap=False)

    def get_pp_transformer_map(self, pp_index):
        return self.pp_to_transformer_map[pp_index]

    def get_transformer_state(self, tp_index, pp_index):
        return [self._merge_state_dicts([load_file(f, mmap=False) for f in files])
                for files in self.transformer_file_map[(tp_index, pp_index)]]

    def get_2d_parallel_state(self, tp_index, pp_index):
        merged = None
        for f in self.get_2d_parallel_files(tp_index=tp_index, pp_index=pp_index):
            sd = load_file(f, mmap=False)
            merged = sd if merged is None else merge_state(merged, sd)
        return merged

    @staticmethod
    def _merge_state_dicts(sd_list):
        """Tensor-parallel merge of one layer's state dicts."""
        first = sd_list[0]
        return {k: (first[k] if k in SEQUENTIAL_LAYERS or len(sd_list) == 1 else
                    torch.cat([sd[k] for sd in sd_list], dim=LAYER_CONCAT_DIM.get(k, 0))) for k in first}

    # ----------------------------------------------------------------------------------------------- maps
    def _build_tp_other_layer_map(self, layer_index):
        if not self.layer_files:
            return {}
        files = get_files_with_prefix(self.layer_files, self.layer_keys[layer_index])
        return dict(enumerate(partition_data(files, self.tp_degree)))

    def _build_pp_transformer_map(self):
        layers = self.layer_keys[1:-1]
        per = len(layers) // self.pp_degree if self.pp_degree else 0
        return {i: layers[i * per:(i + 1) * per] for i in range(self.pp_degree)}

    def _build_transformer_file_map(self):
        layers = self.layer_keys[1:-1]
        per = max(len(layers) // self.pp_degree, 1) if self.pp_degree else 1
        out = {}
        for n, key in enumerate(layers):
            parts = partition_data(get_files_with_prefix(self.layer_files, key), self.tp_degree)
            for t in range(self.tp_degree):
                out.setdefault((t, n // per), []).append(parts[t])
        return out

    def validate_files(self):
        for f in self.file_list:
            if not os.path.isfile(f):
                print(f"Error: {f} is not existent")

    def show_2d_mapping(self):
        for i in range(self.pp_degree):
            for j in range(self.tp_degree):
                print(f"[{i}, {j}] = {self.get_2d_parallel_files(pp_index=i, tp_index=j)}")

    def show_tp_embedding_map(self):
        print(self.tp_to_embedding_map)

    def show_tp_final_norm_map(self):
        print(self.tp_to_final_norm_map)

    def show_pp_transformer_map(self):
        print(self.pp_to_transformer_map)

    def show_transformer_file_map(self):
        print(self.transformer_file_map)
