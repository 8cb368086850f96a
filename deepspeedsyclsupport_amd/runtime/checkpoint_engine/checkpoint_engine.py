"""Pluggable checkpoint writers (reference `runtime/checkpoint_engine/*`: CheckpointEngine ABC, Torch, Nebula).

`AsyncCheckpointEngine` is the MI355X counterpart of the Nebula async engine: state is snapshotted to host memory
(device tensors copied D2H) on the caller's thread, then serialised to disk on a background thread so training
resumes immediately; `commit()` joins outstanding writes.
"""
import os
import threading

import torch

from ...utils.logging import logger


class CheckpointEngine:

    def __init__(self, config_params=None):
        pass

    def create(self, tag):
        pass

    def makedirs(self, path, exist_ok=False):
        os.makedirs(path, exist_ok=exist_ok)

    def save(self, state_dict, path: str):
        raise NotImplementedError

    def load(self, path: str, map_location=None):
        raise NotImplementedError

    def commit(self, tag):
        return True


class TorchCheckpointEngine(CheckpointEngine):

    def save(self, state_dict, path: str):
        torch.save(state_dict, path)

    def load(self, path: str, map_location=None):
        # our checkpoints hold only tensors / containers / primitives (the loss scaler is saved as a dict), so they
        # load with the non-executing loader; reference-written files additionally pickle a few inert objects
        # (LossScaler, fragment_address), matched to allow-listed stand-ins (checkpoint/zero_checkpoint.py)
        from ...checkpoint.zero_checkpoint import _reference_pickle_stubs
        with torch.serialization.safe_globals(_reference_pickle_stubs()):
            return torch.load(path, map_location=map_location, weights_only=True)


def _to_host(obj):
    if torch.is_tensor(obj):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return type(obj)((k, _to_host(v)) for k, v in obj.items()) if not hasattr(obj, "default_factory") else \
            {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    return obj


class AsyncCheckpointEngine(TorchCheckpointEngine):

    def __init__(self, config_params=None):
        super().__init__(config_params)
        self._threads = []

    def save(self, state_dict, path: str):
        snap = _to_host(state_dict)
        t = threading.Thread(target=torch.save, args=(snap, path), daemon=True)
        t.start()
        self._threads.append(t)

    def commit(self, tag):
        for t in self._threads:
            t.join()
        self._threads = []
        logger.info(f"[AsyncCheckpointEngine] checkpoint {tag} is committed")
        return True
