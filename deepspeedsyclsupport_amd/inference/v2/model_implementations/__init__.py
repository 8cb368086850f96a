"""Checkpoint -> model plumbing of inference v2 (reference `inference/v2/model_implementations/`)."""
from . import archs
from .archs import (FalconPolicy, Llama2Policy, MistralPolicy, MixtralPolicy, OPTPolicy, PhiPolicy)
from .inference_model_base import DSInferenceModelBase, MPType
from .inference_policy_base import POLICIES, ContainerMap, InferenceV2Policy
from .inference_transformer_base import DSMoETransformerModelBase, DSTransformerModelBase
from .layer_container_base import LayerContainer
from .parameter_base import ParameterBase, ParamList
