"""Transformer model bases of inference v2 (reference
`inference/v2/model_implementations/inference_transformer_base.py`): the dense and MoE decoders are both
`DSInferenceModel` driven by the spec."""
from ...model_implementations.transformer import DSInferenceModel as DSTransformerModelBase

DSMoETransformerModelBase = DSTransformerModelBase

__all__ = ["DSTransformerModelBase", "DSMoETransformerModelBase"]
