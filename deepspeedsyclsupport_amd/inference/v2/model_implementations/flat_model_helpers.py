"""Serialised form of an injected model (reference `inference/v2/model_implementations/flat_model_helpers.py`):
`flatten_inference_model` writes what `InferenceEngineV2.serialize` writes (the spec as JSON + this rank's tensors as
safetensors), `restore_inference_model` rebuilds the model from those files."""
import dataclasses
import json
import os

import torch


def make_param_filename(base: str, mp_rank: int, mp_size: int) -> str:
    return os.path.join(base, f"params_rank_{mp_rank}.safetensors")


def make_metadata_filename(base: str, mp_rank: int, mp_size: int) -> str:
    return os.path.join(base, "ds_model_meta.json")


def make_model_config_filename(base: str) -> str:
    return os.path.join(base, "ds_model_config.json")


def pad_to_aligned_offset(offset: int, alignment: int = 256) -> int:
    return -(-offset // alignment) * alignment


def flatten_inference_model(model, save_path: str) -> None:
    from safetensors.torch import save_file
    os.makedirs(save_path, exist_ok=True)
    sd = {k: v.detach().contiguous().cpu() for k, v in model.state_dict().items()}
    save_file(sd, make_param_filename(save_path, model.tp_rank, model.tp_size))
    if model.tp_rank == 0:
        with open(make_model_config_filename(save_path), "w") as f:
            json.dump(dataclasses.asdict(model.spec), f)
        with open(make_metadata_filename(save_path, 0, model.tp_size), "w") as f:
            json.dump({"dtype": str(model.dtype).replace("torch.", ""), "tp_size": model.tp_size}, f)


def restore_inference_model(save_path: str, engine_config=None, device=None):
    from ..engine_factory import build_engine_from_ds_checkpoint
    return build_engine_from_ds_checkpoint(save_path, engine_config, device=device).model


_ = torch
