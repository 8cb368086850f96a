"""Policies: how a checkpoint becomes an injected model (reference
`inference/v2/model_implementations/inference_policy_base.py`).

`InferenceV2Policy.build_model` creates the (sharded, device-resident) `DSInferenceModel` for the checkpoint's
config, then streams the checkpoint engine's tensors through a `ContainerMap`: each tensor goes to the container its
name belongs to, and as soon as a transformer layer's container is complete the layer is sliced for this rank,
copied to the device and released. Host memory therefore holds at most the tensors of the layers still incomplete
(and with memory-mapped safetensors not even those).
"""
import re
from abc import ABC, abstractmethod
from typing import Iterable, List, Optional, Union

import torch

from ...model_implementations import convert
from ...model_implementations.transformer import DSInferenceModel
from ..checkpoint.base_engine import CheckpointEngineBase
from .layer_container_base import LayerContainer

POLICIES = {}


class ContainerMap:

    def __init__(self) -> None:
        self._prefix_map = {}         # transformer prefix -> list of containers
        self._transformer_params = None
        self._non_transformer_params = None
        self._unmapped = []

    @property
    def transformer_params(self) -> List[LayerContainer]:
        return self._transformer_params

    @property
    def non_transformer_params(self) -> LayerContainer:
        return self._non_transformer_params

    def set_transformer_params(self, prefixes: Union[str, Iterable[str]], containers: List[LayerContainer]) -> None:
        """`prefixes`: checkpoint prefix(es) of the layer list ("model.layers"): names `<prefix>.<i>.<rest>` go to
        containers[i] as `<rest>`."""
        prefixes = [prefixes] if isinstance(prefixes, str) else list(prefixes)
        self._transformer_params = containers
        self._layer_rx = [re.compile("^" + re.escape(p) + r"\.(\d+)\.(.*)$") for p in prefixes]

    def set_non_transformer_params(self, container: LayerContainer) -> None:
        self._non_transformer_params = container

    def set_unmapped_params(self, names: Union[str, Iterable[str]]) -> None:
        """Checkpoint names (regular expressions) that are deliberately ignored (rotary inv_freq buffers, ...)."""
        names = [names] if isinstance(names, str) else list(names)
        self._unmapped = [re.compile(n) for n in names]

    def map_param(self, name: str, parameter: torch.Tensor) -> Optional[int]:
        """Route one tensor. Returns the layer index it went to (None for non-transformer tensors)."""
        for rx in self._layer_rx:
            m = rx.match(name)
            if m:
                idx = int(m.group(1))
                if idx >= len(self._transformer_params):
                    raise ValueError(f"{name}: layer {idx} is beyond the model's {len(self._transformer_params)}")
                if not self._transformer_params[idx].set_dependency(m.group(2), parameter) \
                        and not self._ignored(name):
                    raise ValueError(f"Cannot find container for {name}, please double check the Containers/"
                                     f"ContainerMap")
                return idx
        if not self._non_transformer_params.set_dependency(name, parameter) and not self._ignored(name):
            raise ValueError(f"Cannot find container for {name}, please double check the Containers/ContainerMap")
        return None

    def _ignored(self, name):
        return any(rx.search(name) for rx in self._unmapped)

    def validate(self) -> None:
        for i, c in enumerate(self._transformer_params):
            if c is not None and not c.is_initialized:
                raise RuntimeError(f"Transformer container {i} not fully initialized after checkpoint load: "
                                   f"missing {c.missing()}")
        if not self._non_transformer_params.is_initialized:
            raise RuntimeError(f"Non-transformer container not fully initialized after checkpoint load: missing "
                               f"{self._non_transformer_params.missing()}")


class _ModelView:
    """What parameters need to know about the model while it loads."""

    def __init__(self, spec):
        self.spec = spec
        self.n_experts = spec.num_experts


class InferenceV2Policy(ABC):
    #: `model_type` values of HF configs this policy serves (registered into POLICIES by `register`)
    model_types = ()

    def __init__(self, model_config, checkpoint_engine: Optional[CheckpointEngineBase] = None,
                 inf_checkpoint_path: Optional[str] = None) -> None:
        if checkpoint_engine is None and inf_checkpoint_path is None:
            raise ValueError("Either checkpoint_engine or inf_checkpoint_path must be specified.")
        self._model_config = model_config
        self._checkpoint_engine = checkpoint_engine
        self._inf_checkpoint_path = inf_checkpoint_path
        self._model = None

    # ------------------------------------------------------------------------------------------ per model
    def spec(self):
        return convert.spec_from_config(self._model_config)

    def instantiate_model(self, engine_config, mp_group=None) -> DSInferenceModel:
        from ...config import to_dtype
        tp = engine_config.tensor_parallel.tp_size
        rank = 0
        if tp > 1:
            from .... import comm as dist
            rank = dist.get_rank(mp_group)
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
            torch.device("cpu")
        spec = self.spec()
        spec.max_positions = max(spec.max_positions, engine_config.state_manager.max_context)
        dtype = to_dtype(getattr(self, "dtype", None) or torch.bfloat16)
        return DSInferenceModel(spec, mp_group, tp, rank, dtype, device)

    @abstractmethod
    def build_container_map(self) -> ContainerMap:
        ...

    # ------------------------------------------------------------------------------------------ build
    def build_model(self, engine_config, mp_group=None) -> DSInferenceModel:
        if self._checkpoint_engine is None:
            from ..engine_factory import build_engine_from_ds_checkpoint
            return build_engine_from_ds_checkpoint(self._inf_checkpoint_path, engine_config).model
        self.model = model = self.instantiate_model(engine_config, mp_group)
        self._view = _ModelView(model.spec)
        cmap = self.build_container_map()
        with torch.no_grad():
            for name, tensor in self._checkpoint_engine.parameters():
                idx = cmap.map_param(name, tensor)
                if idx is not None:
                    c = cmap.transformer_params[idx]
                    if c is not None and self._layer_done(c):
                        convert.load_layer(model, idx, self._finish_layer(c.canonical()))
                        c.release()
                        cmap.transformer_params[idx] = None
            for i, c in enumerate(cmap.transformer_params):   # layers whose optional tensors never came
                if c is not None and c.is_initialized:
                    convert.load_layer(model, i, self._finish_layer(c.canonical()))
                    c.release()
                    cmap.transformer_params[i] = None
            cmap.validate()
            top = cmap.non_transformer_params.canonical()
            if "lm_head" not in top:      # tied embeddings
                top["lm_head"] = top["embed"]
            convert.load_top(model, self._finish_top(top))
        return model

    def _layer_done(self, container) -> bool:
        """All tensors the layer is expected to have are present (every mapped field, not merely every touched
        parameter: a layer is loaded once, when nothing more can arrive)."""
        return all(p.complete for p in container._params.values() if not getattr(p, "optional", False))

    def _finish_layer(self, lw):
        return lw

    def _finish_top(self, top):
        return top


def register(policy_cls):
    for mt in policy_cls.model_types:
        POLICIES[mt] = policy_cls
    return policy_cls


PolicyMeta = type(InferenceV2Policy)
