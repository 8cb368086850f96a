"""Op-level inference transformer layers (reference `ops/transformer/inference/__init__.py`): the standalone fused
decoder layer a user can drop into their own model, its config, the MoE variant and the diffusers blocks.

The compute is the same as the kernel-injected inference path (`inference/model_implementations/transformer.py`
`DSInferenceLayer`: fused norm + QKV epilogue with RoPE and paged-KV append, flash prefill / paged decode attention,
skinny weight-streaming GEMMs for decode); this package only gives it the reference's op-level API."""
from .config import DeepSpeedInferenceConfig, DeepSpeedMoEInferenceConfig  # noqa: F401
from .layer import DeepSpeedTransformerInference, DeepSpeedMoEInference  # noqa: F401
from ....module_inject.diffusers import DSDiffusersAttention as DeepSpeedDiffusersAttention  # noqa: F401
from ....module_inject.diffusers import DSDiffusersTransformerBlock as DeepSpeedDiffusersTransformerBlock  # noqa: F401
