"""Hugging Face checkpoint directory as a parameter stream (reference
`inference/v2/checkpoint/huggingface_engine.py`).

Local directories only (this build never fetches). Safetensors shards are opened with `safe_open`, so each tensor is
a memory-mapped view that costs page cache, not anonymous host memory, until it is copied to the device; `.bin`
shards are loaded with `torch.load(weights_only=True, mmap=True)`.
"""
import json
import os

import torch

from .base_engine import CheckpointEngineBase


class HuggingFaceCheckpointEngine(CheckpointEngineBase):

    def __init__(self, model_name_or_path: str, auth_token: str = None) -> None:
        super().__init__()
        if not os.path.isdir(model_name_or_path):
            raise FileNotFoundError(f"{model_name_or_path} is not a local checkpoint directory (checkpoints are "
                                    f"never downloaded)")
        self.model_name_or_path = model_name_or_path
        from transformers import AutoConfig, GenerationConfig
        self.model_config = AutoConfig.from_pretrained(model_name_or_path, local_files_only=True)
        try:
            self.generation_config = GenerationConfig.from_pretrained(model_name_or_path, local_files_only=True)
        except Exception:
            self.generation_config = None
        self._files = self._shards()

    def _shards(self):
        d = self.model_name_or_path
        for index, single in (("model.safetensors.index.json", "model.safetensors"),
                              ("pytorch_model.bin.index.json", "pytorch_model.bin")):
            ip = os.path.join(d, index)
            if os.path.exists(ip):
                with open(ip) as f:
                    names = sorted(set(json.load(f)["weight_map"].values()))
                return [os.path.join(d, n) for n in names]
            if os.path.exists(os.path.join(d, single)):
                return [os.path.join(d, single)]
        raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin (or their index files) in {d}")

    def parameters(self):
        for path in self._files:
            if path.endswith(".safetensors"):
                from safetensors import safe_open
                with safe_open(path, framework="pt", device="cpu") as f:
                    for name in f.keys():
                        yield name, f.get_tensor(name)
            else:
                sd = torch.load(path, map_location="cpu", weights_only=True, mmap=True)
                for name in list(sd.keys()):
                    yield name, sd.pop(name)
