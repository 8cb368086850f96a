"""Kernel injection and automatic tensor parallelism (reference `deepspeed/module_inject/`)."""
from .auto_tp import AutoTP
from .layers import EmbeddingLayer, LinearAllreduce, LinearLayer, LmHeadLinearAllreduce, Normalize, RMSNormalize
from .replace_module import ReplaceWithTensorSlicing, generic_injection, replace_transformer_layer, \
    revert_transformer_layer
