"""Model-parallel re-sharding of Megatron checkpoints at load time (reference `runtime/state_dict_factory.py:21`
`SDLoaderFactory`, `:47` `SDLoaderBase`, `:185` `MegatronSDLoader`).

A checkpoint written at model-parallel degree P (files `mp_rank_00 .. P-1`) is served to a job at degree M:
  * M == P: rank r reads file r (optionally int8-quantised on the way in);
  * M <  P: rank r concatenates files [r*P/M, (r+1)*P/M) — merge;
  * M >  P: rank r slices its piece out of file r*P/M — split.
Each Megatron weight is sharded along a known axis, so one rule table drives both directions:

    rule       keys                                                     axis
    COL        attention.dense.weight, mlp.dense_4h_to_h.weight         1  (row-parallel: input dim split)
    ROW        mlp.dense_h_to_4h.{weight,bias}, word_embeddings.weight, 0  (column-parallel: output dim split)
               final_linear.weight (split only, as in the reference)
    QKV        attention.query_key_value.{weight,bias}                  0, version-dependent packing
    REPLICATE  everything else (norms, biases of row-parallel layers, position embeddings)

Megatron packs the fused QKV three ways (checkpoint_version): 0 = [3, heads, hn] (q block, k block, v block — each
shard carries its own three blocks, so merging/splitting works per block), 1.0 = [heads, hn, 3] and
2.0 = [heads, 3, hn] (head-major: a plain concatenation / slice along dim 0).

`bloom` / `ds_model` descriptors (HF-layout shards listed in a JSON) are returned as-is for the inference engine,
which streams them into the model one file at a time.

Files load through the checkpoint engine's non-executing loader (`torch.load(weights_only=True)`).
"""
import collections
import copy
import json
import os
from abc import ABC, abstractmethod

import torch

from ..utils.logging import logger
from .checkpoint_engine import TorchCheckpointEngine
from .weight_quantizer import WeightQuantization

AUTO_MODULE_KEY = "auto"

COL, ROW, QKV, REPLICATE = "col", "row", "qkv", "replicate"
_RULES = (
    (QKV, ("attention.query_key_value", )),
    (COL, ("attention.dense.weight", "mlp.dense_4h_to_h.weight")),
    (ROW, ("mlp.dense_h_to_4h.weight", "mlp.dense_h_to_4h.bias", "word_embeddings.weight")),
)
_SPLIT_ONLY_ROW = ("final_linear.weight", )
_QUANTIZED = ("attention.query_key_value.weight", "attention.dense.weight", "mlp.dense_h_to_4h.weight",
              "mlp.dense_4h_to_h.weight")


def shard_rule(key, splitting=False):
    for rule, pats in _RULES:
        if any(p in key for p in pats):
            return rule
    if splitting and any(p in key for p in _SPLIT_ONLY_ROW):
        return ROW
    return REPLICATE


class SDLoaderFactory:

    @staticmethod
    def get_sd_loader_json(json_file, checkpoint_engine=None):
        if isinstance(json_file, str):
            with open(json_file) as f:
                data = json.load(f)
        else:
            assert isinstance(json_file, dict), "checkpoint descriptor must be a JSON path or a dict"
            data = json_file
        sd_type = data["type"]
        if sd_type.lower() in ("bloom", "ds_model"):
            return data
        return SDLoaderFactory.get_sd_loader(data["checkpoints"], checkpoint_engine, sd_type, data.get("version"))

    @staticmethod
    def get_sd_loader(ckpt_list, checkpoint_engine=None, sd_type="Megatron", version=None):
        if sd_type != "Megatron":
            raise ValueError(f"{sd_type} checkpoint type is not supported")
        return MegatronSDLoader(ckpt_list, version, checkpoint_engine)


class SDLoaderBase(ABC):

    def __init__(self, ckpt_list, version, checkpoint_engine=None):
        self.module_key = None
        self.ckpt_list = list(ckpt_list)
        self.version = version
        self.checkpoint_engine = checkpoint_engine or TorchCheckpointEngine()
        self.check_ckpt_list()

    def _load(self, path):
        return self.checkpoint_engine.load(path, map_location="cpu")

    def load(self, mp_world_size, mp_rank, module_key=AUTO_MODULE_KEY, is_pipe_parallel=False, quantize=False,
             quantize_bits=8, quantize_groups=64, mlp_extra_grouping=True):
        """-> (path of the primary file, state dict for this mp rank, (int8 scale table or None, merge count))."""
        self.module_key = module_key
        n = len(self.ckpt_list)
        idx = mp_rank * n // mp_world_size
        if is_pipe_parallel and module_key is not None and mp_world_size != n:
            # pipeline mp_rank_* files under a degree change hold identical copies: read the first
            mp_world_size, idx = n, 0
        path = self.ckpt_list[idx]
        if n == mp_world_size:
            sd = self._load(path)
            scales = None
            if quantize:
                wq = WeightQuantization(mlp_extra_grouping=mlp_extra_grouping, mp_size=mp_world_size)
                module, scales = wq.sd_quantize_megatron(self.get_module(sd), quantize_bits, quantize_groups)
                sd = self.set_module(sd, module)
            return path, sd, (scales, 1)
        if n > mp_world_size:
            sd, scales, count = self.merge_state_dict(mp_world_size, mp_rank, quantize, quantize_bits,
                                                      quantize_groups, mlp_extra_grouping)
            return path, sd, (scales, count)
        sd, scales = self.split_state_dict(mp_world_size, mp_rank, quantize, quantize_bits, quantize_groups,
                                           mlp_extra_grouping)
        return path, sd, (scales, 1)

    def get_merge_state_dicts(self, mp_world_size, mp_rank):
        n = len(self.ckpt_list)
        if n % mp_world_size:
            raise ValueError(f"cannot merge {n} checkpoint files onto model-parallel degree {mp_world_size}")
        k = n // mp_world_size
        files = self.ckpt_list[k * mp_rank:k * (mp_rank + 1)]
        logger.info(f"mp_rank {mp_rank}: merging {files}")
        return [self._load(f) for f in files]

    def get_split_state_dict(self, mp_world_size, mp_rank):
        n = len(self.ckpt_list)
        if mp_world_size % n:
            raise ValueError(f"cannot split {n} checkpoint files onto model-parallel degree {mp_world_size}")
        per_file = mp_world_size // n
        idx, offset = divmod(mp_rank, per_file)
        logger.info(f"mp_rank {mp_rank}: slice {offset}/{per_file} of {self.ckpt_list[idx]}")
        return self._load(self.ckpt_list[idx]), per_file, offset

    @staticmethod
    def _choose_module_key(sd):
        if "module" in sd and "model" in sd:
            raise ValueError("checkpoint has both 'model' and 'module' keys")
        if "module" in sd:
            return "module"
        if "model" in sd:
            return "model"
        raise ValueError("checkpoint contains neither 'model' nor 'module'")

    def get_module(self, sd):
        if self.module_key is None:
            return sd
        return sd[self._choose_module_key(sd) if self.module_key == AUTO_MODULE_KEY else self.module_key]

    def set_module(self, sd, module):
        if self.module_key is None:
            return module
        sd[self._choose_module_key(sd) if self.module_key == AUTO_MODULE_KEY else self.module_key] = module
        return sd

    def check_ckpt_list(self):
        if not self.ckpt_list:
            raise ValueError("empty checkpoint list")
        sd = self._load(self.ckpt_list[0])
        if "mp_world_size" in sd and len(self.ckpt_list) != sd["mp_world_size"]:
            raise ValueError(f"{len(self.ckpt_list)} checkpoint files but the checkpoint was saved at "
                             f"mp_world_size={sd['mp_world_size']}")

    @abstractmethod
    def merge_state_dict(self, mp_world_size, mp_rank, quantize, quantize_bits, groups, mlp_extra_grouping):
        ...

    @abstractmethod
    def split_state_dict(self, mp_world_size, mp_rank, quantize, quantize_bits, groups, mlp_extra_grouping):
        ...

    @abstractmethod
    def sanity_check(self, ckpt_file_name):
        ...


class MegatronSDLoader(SDLoaderBase):

    # ------------------------------------------------------------------------------------------ fused QKV
    @staticmethod
    def merge_query_key_value(param_list, ckpt_ver):
        if ckpt_ver == 0:
            # each shard is [q_i; k_i; v_i]: gather the q blocks of all shards, then k, then v
            blocks = [torch.chunk(p, 3, dim=0) for p in param_list]
            return torch.cat([torch.cat([b[j] for b in blocks], dim=0) for j in range(3)], dim=0)
        if ckpt_ver in (1.0, 2.0):
            return torch.cat(param_list, dim=0)
        raise ValueError(f"checkpoint version {ckpt_ver} is not supported")

    @staticmethod
    def split_query_key_value(param, num_to_split, offset, ckpt_ver):
        if ckpt_ver == 0:
            return torch.cat([torch.chunk(b, num_to_split, dim=0)[offset] for b in torch.chunk(param, 3, dim=0)],
                             dim=0)
        if ckpt_ver in (1.0, 2.0):
            return torch.chunk(param, num_to_split, dim=0)[offset]
        raise ValueError(f"checkpoint version {ckpt_ver} is not supported")

    def get_checkpoint_version(self, state_dict):
        return self.version if self.version is not None else state_dict.get("checkpoint_version", 0)

    # ------------------------------------------------------------------------------------------ merge / split
    def merge_state_dict(self, mp_world_size, mp_rank, quantize=False, quantize_bits=8, groups=64,
                         mlp_extra_grouping=True):
        self.sanity_check(self.ckpt_list[0])
        sds = self.get_merge_state_dicts(mp_world_size, mp_rank)
        out = copy.deepcopy(sds[0])
        modules = [self.get_module(sd) for sd in sds]
        ver = self.get_checkpoint_version(out)
        wq = WeightQuantization(mlp_extra_grouping=mlp_extra_grouping, mp_size=mp_world_size) if quantize else None
        merged = collections.OrderedDict()
        for key in modules[0].keys():
            vals = [m[key] for m in modules]
            rule = shard_rule(key)
            q = wq is not None and any(p in key for p in _QUANTIZED)
            if rule == COL:
                merged[key] = torch.cat(wq.Quantize(vals, quantize_bits, groups, key=key, merge_dim=1) if q else vals,
                                        dim=1)
            elif rule == QKV:
                # quantised QKV keeps the per-shard packing (the scales follow the same shard order)
                merged[key] = torch.cat(wq.Quantize(vals, quantize_bits, groups, key=key), dim=0) if q else \
                    (torch.cat(vals, dim=0) if wq is not None else self.merge_query_key_value(vals, ver))
            elif rule == ROW:
                merged[key] = torch.cat(wq.Quantize(vals, quantize_bits, groups, key=key) if q else vals, dim=0)
            else:
                merged[key] = vals[0]
        return self.set_module(out, merged), (wq.merge_scales() if wq is not None else None), len(modules)

    def split_state_dict(self, mp_world_size, mp_rank, quantize=False, quantize_bits=8, groups=64,
                         mlp_extra_grouping=True):
        sd, per_file, offset = self.get_split_state_dict(mp_world_size, mp_rank)
        out = copy.deepcopy(sd)
        module = self.get_module(sd)
        ver = self.get_checkpoint_version(out)
        wq = WeightQuantization(mlp_extra_grouping=mlp_extra_grouping, mp_size=mp_world_size) if quantize else None
        split = collections.OrderedDict()
        for key, val in module.items():
            rule = shard_rule(key, splitting=True)
            if wq is not None and any(p in key for p in _QUANTIZED):
                val = wq.Quantize([val], quantize_bits, groups, key)[0]
            if rule == COL:
                if val.shape[1] % per_file:
                    raise ValueError(f"{key}: dim 1 ({val.shape[1]}) not divisible by {per_file}")
                split[key] = torch.chunk(val, per_file, dim=1)[offset]
            elif rule == QKV:
                split[key] = self.split_query_key_value(val, per_file, offset, ver)
            elif rule == ROW:
                if val.shape[0] % per_file:
                    raise ValueError(f"{key}: dim 0 ({val.shape[0]}) not divisible by {per_file}")
                split[key] = torch.chunk(val, per_file, dim=0)[offset]
            else:
                split[key] = val
        scales = wq.merge_scales_split(per_file) if wq is not None else None
        return self.set_module(out, split), scales

    def sanity_check(self, ckpt_file_name):
        module = self.get_module(self._load(ckpt_file_name))
        for must in ("attention.dense.weight", "mlp.dense_4h_to_h.weight", "attention.query_key_value",
                     "mlp.dense_h_to_4h.weight", "mlp.dense_h_to_4h.bias"):
            if not any(must in k for k in module.keys()):
                raise ValueError(f"key {must} is not found in the checkpoint {ckpt_file_name}")


def load_hf_shards(model, descriptor, base_dir="", device="cpu"):
    """Stream the shard files of a `bloom` / `ds_model` descriptor into `model` one file at a time (a meta-device
    model gets its tensors assigned from the files; nothing else is materialised). Returns the keys loaded."""
    files = descriptor["checkpoints"]
    if isinstance(files, dict):  # {"non_tp": [...], "tp": [...]} layout of pre-sharded ds_model checkpoints
        files = list(files.get("non_tp", [])) + list(files.get("tp", []))
    base = descriptor.get("base_dir") or base_dir or ""
    loaded = set()
    for f in files:
        path = f if os.path.isabs(f) else os.path.join(base, f)
        if path.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(path, device="cpu")
        else:
            sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = sd.get("module", sd) if isinstance(sd, dict) else sd
        missing_ok = model.load_state_dict(sd, strict=False, assign=True)
        loaded.update(k for k in sd.keys() if k not in missing_ok.unexpected_keys)
        del sd
    return loaded
