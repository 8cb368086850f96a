"""Dense pointwise / normalisation / GEMM kernel objects of inference v2 (reference
`inference/v2/kernels/core_ops/{bias_activations,blas_kernels,cuda_layer_norm,cuda_rms_norm,gated_activations}`).

Each object validates its configuration at construction and is then called with caller-owned output tensors, as in
the reference. The work runs in the gfx950 kernels behind `ops/transformer/functional.py` (`act_kernels.hip`,
`norm_kernels.hip`: a block per row from 1024 channels, fused residual add) and the library GEMM; on a CPU tensor the
same functions fall back to torch, which is what the CPU tests compare against.

Layout note: the gated activation takes the gate half and the linear half side by side ([.., gate | up]) — the layout
`GatedMLPParameter` produces here — not interleaved element pairs.
"""
from typing import Optional

import torch

from ....ops.transformer import functional as DF
from ..inference_utils import ActivationType, DtypeEnum, act_name, elem_size
from .ds_kernel import DSKernelBase

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`


def _dtype(dt):
    return dt.value if isinstance(dt, DtypeEnum) else DtypeEnum(dt).value


def _check_dtype(dt, allowed, what="data type"):
    t = _dtype(dt)
    if t not in [_dtype(a) for a in allowed]:
        raise ValueError(f"Unsupported {what}: {dt}, supported_dtypes are {allowed}")
    return t


def _into(out, value):
    if out.data_ptr() != value.data_ptr():
        out.copy_(value.view(out.shape))
    return out


class CUDABiasActivation(DSKernelBase):
    """activation = act(activation + bias), in place."""
    supported_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16]
    supported_act_fns = [ActivationType.IDENTITY, ActivationType.GELU, ActivationType.RELU, ActivationType.SILU]

    def __init__(self, channels: int, dtype: DtypeEnum, act_fn: ActivationType) -> None:
        if channels % 8 != 0:
            raise ValueError("channels must be divisible by 8")
        self.dtype = _check_dtype(dtype, self.supported_dtypes)
        act_fn = ActivationType(act_fn)
        if act_fn not in self.supported_act_fns:
            raise ValueError(f"Unsupported activation function: {act_fn}, supported_act_fns are "
                             f"{self.supported_act_fns}")
        self.channels, self.act = channels, act_name(act_fn)

    def __call__(self, activation: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.act == "identity":
            if bias is not None:
                activation.add_(bias)
            return activation
        return _into(activation, DF.bias_activation(activation, bias, self.act))


class BlasLibLinear(DSKernelBase):
    """output = hidden_states . weights^T (weights [out, in], or [batch, out, in] for a batched product)."""
    supported_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16, DtypeEnum.fp32]

    def __init__(self, fp_dtype: DtypeEnum):
        self.dtype = _check_dtype(fp_dtype, self.supported_dtypes)

    def __call__(self, output: torch.Tensor, hidden_states: torch.Tensor, weights: torch.Tensor) -> torch.Tensor:
        torch.matmul(hidden_states, weights.transpose(-1, -2), out=output)
        return output


class CUDAFPLNBase(DSKernelBase):
    supported_dtypes = [torch.float16, torch.bfloat16, torch.float32]

    def __init__(self, channels: int, fp_dtype: torch.dtype, epsilon: float = 1e-5):
        self.dtype = _check_dtype(fp_dtype, self.supported_dtypes)
        if (channels * elem_size(self.dtype)) % 16 != 0:
            raise ValueError("channels must be divisible by 16 bytes")
        self.channels, self.epsilon = channels, epsilon


class CUDAFPLN(CUDAFPLNBase):
    """output_z = LayerNorm(input_x)."""

    def __call__(self, output_z, input_x, gamma, beta):
        return _into(output_z, DF.layer_norm(input_x, gamma, beta, self.epsilon))


class CUDAFPPostLN(CUDAFPLNBase):
    """output_z = LayerNorm(input_x + input_y) (post-norm residual)."""

    def __call__(self, output_z, input_x, input_y, gamma, beta):
        y, _ = DF.layer_norm(input_x, gamma, beta, self.epsilon, input_y)
        return _into(output_z, y)


class CUDAFPPreLN(CUDAFPLNBase):
    """z_res = x_res + y_hid; z_hid = LayerNorm(z_res) (pre-norm residual stream)."""

    def __call__(self, z_res, z_hid, x_res, y_hid, gamma, beta):
        y, res = DF.layer_norm(y_hid, gamma, beta, self.epsilon, x_res)
        return _into(z_res, res), _into(z_hid, y)


class CUDARMSNormBase(DSKernelBase):
    supported_dtypes = [torch.float16, torch.bfloat16, torch.float32]

    def __init__(self, channels: int, fp_dtype: torch.dtype, epsilon: float = 1e-5):
        self.dtype = _check_dtype(fp_dtype, self.supported_dtypes)
        if (channels * elem_size(self.dtype)) % 16 != 0:
            raise ValueError("channels must be divisible by 16 bytes")
        self.channels, self.epsilon = channels, epsilon


class CUDARMSNorm(CUDARMSNormBase):
    """output_z = RMSNorm(input_x)."""

    def __call__(self, output_z, input_x, gamma):
        return _into(output_z, DF.rms_norm(input_x, gamma, self.epsilon))


class CUDARMSPreNorm(CUDARMSNormBase):
    """z_res = x_res + y_hid; z_hid = RMSNorm(z_res)."""

    def __call__(self, z_res, z_hid, x_res, y_hid, gamma):
        y, res = DF.rms_norm(y_hid, gamma, self.epsilon, x_res)
        return _into(z_res, res), _into(z_hid, y)


class CUDAGatedActivation(DSKernelBase):
    """output[.., c] = act(input[.., c] + bias[c]) * (input[.., C + c] + bias[C + c]), C = channels."""
    supported_dtypes = [torch.float16, torch.bfloat16, torch.float32]
    supported_act_fns = [ActivationType.GEGLU, ActivationType.ReGLU, ActivationType.SiGLU]

    def __init__(self, channels: int, fp_dtype: torch.dtype, act_fn: ActivationType) -> None:
        self.dtype = _check_dtype(fp_dtype, self.supported_dtypes)
        act_fn = ActivationType(act_fn)
        if act_fn not in self.supported_act_fns:
            raise ValueError(f"Unsupported activation function: {act_fn}, supported_act_fns are "
                             f"{self.supported_act_fns}")
        if (channels * elem_size(self.dtype)) % 16 != 0:
            raise ValueError("Channels must be divisible by 16 bytes")
        self.channels, self.act = channels, act_name(act_fn)

    def __call__(self, output: torch.Tensor, input: torch.Tensor, bias: Optional[torch.Tensor] = None) -> None:
        if input.shape[-1] != 2 * self.channels:
            raise ValueError(f"input holds {input.shape[-1]} channels, expected 2 x {self.channels}")
        if bias is not None:
            input = input + bias
        _into(output, DF.gated_activation(input, self.act))
