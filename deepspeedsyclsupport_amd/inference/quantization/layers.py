"""Drop-in quantised `nn.Linear` / `nn.Embedding` (reference `inference/quantization/layers.py:48-114`).

The packed codes and their (scale, minimum) pairs are buffers of the module, so `.to()`, `state_dict()` and HIP-graph
capture treat them like any other tensor. The linear dequantises its weight into a temporary and calls the plain GEMM
(never the ZeRO-3 linear function, which would keep the temporary alive); the embedding dequantises only the rows that
were looked up. Modules that shared one weight before quantisation (tied input embedding / LM head) share one set of
codes after it.
"""
from typing import Dict

import torch
from torch import Tensor, nn
from torch.nn import functional as F

from .utils import DeQuantizer, Packed, Quantizer

quantized_weight_registry = {}  # id(original weight) -> (codes, scale, minimum, shape, moved); cleared after a pass


def _full_weight(layer):
    """The layer's weight as a whole tensor: a ZeRO-3 partitioned parameter is gathered for the moment of reading."""
    w = layer.weight
    if hasattr(w, "ds_id"):
        from ...runtime.zero.partition_parameters import GatheredParameters
        with GatheredParameters([w]):
            return w.detach().clone()
    return w.detach()


class _QuantizedWeight:
    """Mixin: owns `q_codes`, `q_scale`, `q_min` buffers and rebuilds the weight from them."""

    def _adopt(self, config: Dict, pre_quant_layer: nn.Module):
        self.config = config
        key = id(pre_quant_layer.weight)
        if key not in quantized_weight_registry:
            w = _full_weight(pre_quant_layer)
            packed, scale, minimum = Quantizer(config).quantize(w)
            quantized_weight_registry[key] = (packed.data, scale, minimum, packed.shape, packed.moved)
        codes, scale, minimum, shape, moved = quantized_weight_registry[key]
        self.register_buffer("q_codes", codes)
        self.register_buffer("q_scale", scale)
        self.register_buffer("q_min", minimum)
        self._q_shape, self._q_moved = shape, moved
        self.dequantizer = DeQuantizer(config, pre_quant_layer.weight.dtype)

    def _packed(self):
        return Packed(self.q_codes, self._q_shape, self._q_moved)

    def dequantized_weight(self) -> Tensor:
        return self.dequantizer.dequantize(self._packed(), self.q_scale, self.q_min)

    def quantized_nbytes(self):
        return sum(t.numel() * t.element_size() for t in (self.q_codes, self.q_scale, self.q_min))


class QuantizedLinear(nn.Module, _QuantizedWeight):

    def __init__(self, config: Dict, pre_quant_layer: nn.Linear) -> None:
        super().__init__()
        self.in_features, self.out_features = pre_quant_layer.in_features, pre_quant_layer.out_features
        self.bias = pre_quant_layer.bias
        self._adopt(config, pre_quant_layer)

    def forward(self, input: Tensor) -> Tensor:
        return torch._C._nn.linear(input, self.dequantized_weight(), self.bias)

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}, "
                f"bits={self.config['num_bits']}, group_size={self.config['group_size']}")


class QuantizedEmbedding(nn.Module, _QuantizedWeight):

    def __init__(self, config: Dict, pre_quant_layer: nn.Embedding) -> None:
        super().__init__()
        assert pre_quant_layer.max_norm is None, "Not supported"
        assert pre_quant_layer.norm_type == 2, "Not supported"
        assert not pre_quant_layer.scale_grad_by_freq, "Not supported"
        assert not pre_quant_layer.sparse, "Not supported"
        self.num_embeddings, self.embedding_dim = pre_quant_layer.num_embeddings, pre_quant_layer.embedding_dim
        self.padding_idx = pre_quant_layer.padding_idx
        self._adopt(config, pre_quant_layer)

    def forward(self, input: Tensor) -> Tensor:
        if not self._q_moved:
            return self.dequantizer.dequantize_rows(self._packed(), self.q_scale, self.q_min, input)
        return F.embedding(input, self.dequantized_weight(), self.padding_idx)

    def extra_repr(self):
        return (f"{self.num_embeddings}, {self.embedding_dim}, bits={self.config['num_bits']}, "
                f"group_size={self.config['group_size']}")


QUANTIZATION_LAYER_MAPPINGS = {
    nn.Linear: QuantizedLinear,
    nn.Embedding: QuantizedEmbedding,
}
