"""Inference: v1 kernel-injected engine (`init_inference`) and the v2 ragged-batching engine."""
from .config import DeepSpeedInferenceConfig
from .engine import InferenceEngine
