"""An instantiated model as a parameter stream (reference `inference/v2/checkpoint/in_memory_engine.py`)."""
import torch

from .base_engine import CheckpointEngineBase


class InMemoryModelEngine(CheckpointEngineBase):

    def __init__(self, model: torch.nn.Module) -> None:
        super().__init__()
        self.model = model
        self.model_config = getattr(model, "config", None)

    def parameters(self):
        seen = set()
        for name, t in self.model.state_dict().items():
            if t.data_ptr() in seen and t.numel():   # tied weights appear once
                continue
            seen.add(t.data_ptr())
            yield name, t
