"""Group-wise asymmetric int4 / int8 weight codec (reference `inference/quantization/utils.py:43-158`).

A config is `{"num_bits": 4 | 8, "group_size": g, "group_dim": d, "symmetric": False}`: along dimension `d` every run
of `g` elements shares one (scale, minimum) pair, `x ~ q * scale + minimum` with q in [0, 2^bits - 1].

Device tensors go through the gfx950 group quantiser (`ops/csrc/quant/quant_kernels.hip`, one pass, 16-byte loads,
int4 packed two per byte in-kernel); the groups of those kernels run along the innermost dimension, so a tensor
grouped along another dimension is stored transposed (`Packed.moved`). Host tensors use the same math in PyTorch.
Note the scale convention: `scale` here multiplies the code (the reference keeps its reciprocal).
"""
from dataclasses import dataclass
from typing import Dict, Tuple

import torch
from torch import Tensor, nn

from ...ops.quantizer import quantizer as Q


def _check(config: Dict):
    assert config["num_bits"] in (4, 8), "Only INT4 and INT8 quantization is supported."
    assert config["symmetric"] is False, "Only asymmetric quantization is supported at this moment."


@dataclass
class Packed:
    """What `Quantizer.quantize` returns as its first element: the codes plus what is needed to undo the layout."""
    data: Tensor            # int8 storage (int4: two codes per byte), flat, groups along the innermost dimension
    shape: torch.Size       # logical shape of the original tensor
    moved: bool             # True when group_dim was swapped with the last dimension before packing

    def view(self, *a, **k):  # the reference views its packed tensor as other dtypes when handing it around
        return self

    def to(self, *a, **k):
        return Packed(self.data.to(*a, **k), self.shape, self.moved)

    @property
    def nbytes(self):
        return self.data.numel() * self.data.element_size()


class Quantizer:

    def __init__(self, config: Dict) -> None:
        _check(config)
        self.config = config

    def quantize(self, tensor: Tensor) -> Tuple[Packed, Tensor, Tensor]:
        """-> (packed codes, scale [groups], minimum [groups])."""
        c = self.config
        d = c["group_dim"] % tensor.dim()
        assert tensor.shape[d] % c["group_size"] == 0, f"Tensor shape: {tensor.shape} quantization config {c}"
        moved = d != tensor.dim() - 1
        t = tensor.transpose(d, -1) if moved else tensor
        qt = Q.quantize(t.contiguous(), c["group_size"], c["num_bits"], symmetric=False)
        return Packed(qt.data, tensor.shape, moved), qt.scales, qt.zeros


class DeQuantizer:

    def __init__(self, config: Dict, dtype: torch.dtype) -> None:
        _check(config)
        self.config = config
        self.dtype = dtype

    def dequantize(self, tensor: Packed, quant_scale: Tensor, quant_min: Tensor) -> Tensor:
        c = self.config
        d = c["group_dim"] % len(tensor.shape)
        shape = list(tensor.shape)
        if tensor.moved:
            shape[d], shape[-1] = shape[-1], shape[d]
        qt = Q.QuantizedTensor(tensor.data, quant_scale, quant_min, torch.Size(shape), c["group_size"], c["num_bits"],
                               self.dtype)
        out = Q.dequantize(qt, self.dtype)
        return out.transpose(d, -1) if tensor.moved else out

    def dequantize_rows(self, tensor: Packed, quant_scale: Tensor, quant_min: Tensor, rows: Tensor) -> Tensor:
        """Rows `rows` (any shape of indices) of a 2-D tensor grouped along its last dimension, without touching the
        rest of the table: gather the rows' codes and (scale, minimum) pairs, then one dequantise pass over them."""
        c = self.config
        n_rows, width = tensor.shape
        assert not tensor.moved, "row gather needs groups along the embedding dimension"
        per_byte = 2 if c["num_bits"] == 4 else 1
        idx = rows.reshape(-1)
        codes = tensor.data.view(n_rows, width // per_byte).index_select(0, idx)
        gpr = width // c["group_size"]
        s = quant_scale.view(n_rows, gpr).index_select(0, idx).reshape(-1)
        m = quant_min.view(n_rows, gpr).index_select(0, idx).reshape(-1)
        qt = Q.QuantizedTensor(codes.reshape(-1), s, m, torch.Size((idx.numel(), width)), c["group_size"],
                               c["num_bits"], self.dtype)
        return Q.dequantize(qt, self.dtype).view(*rows.shape, width)


def recursive_setattr(model: nn.Module, module_name: str, module: nn.Module):
    """`setattr(model, "a.b.c", module)` through the dotted path."""
    *path, leaf = module_name.split(".")
    for p in path:
        model = getattr(model, p)
    setattr(model, leaf, module)
