"""Checkpoint file names per rank and tensor cloning for compact saves (reference `checkpoint/utils.py:11-62`)."""
import os

import torch

from . import constants as CK


def get_model_ckpt_name_for_rank(base_folder, mp_rank_str):
    return os.path.join(base_folder, f"{CK.MODEL_FILE_PREFIX}{mp_rank_str}{CK.MODEL_FILE_SUFFIX}")


def get_zero_ckpt_name_for_rank(base_folder, dp_rank, mp_rank):
    return os.path.join(base_folder, f"{CK.ZERO_FILE_PREFIX}{dp_rank}_{CK.MODEL_FILE_PREFIX}{mp_rank:02d}"
                        f"{CK.OPTIM_FILE_SUFFIX}")


def get_layer_ckpt_name_for_rank(base_folder, layer_id, tp_rank):
    return os.path.join(base_folder, f"{layer_id}-model_{tp_rank:02d}{CK.MODEL_FILE_SUFFIX}")


def clone_tensors_for_torch_save(item, device=torch.device("cpu")):
    """Copy of a (nested) state with every tensor cloned onto `device`: `torch.save` of a view writes the WHOLE
    underlying storage (a slice of a flat ZeRO buffer would drag the buffer along); clones own exactly their bytes."""
    if torch.is_tensor(item):
        return item.detach().clone().to(device)
    if isinstance(item, (list, tuple)):
        return type(item)(clone_tensors_for_torch_save(v, device) for v in item)
    if isinstance(item, dict):
        return type(item)((k, clone_tensors_for_torch_save(v, device)) for k, v in item.items())
    return item
