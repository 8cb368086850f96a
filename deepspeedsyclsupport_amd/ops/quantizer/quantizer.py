"""Group-wise quantisation front-end (reference `deepspeed/ops/quantizer/quantizer.py:14` ds_quantizer and the
`quantizer` op bindings `csrc/quantization/pt_binding.cpp:270-297`).

Device tensors run the gfx950 kernels (`quant_kernels.hip`); host tensors use the equivalent PyTorch math (also
the numerics oracle in tests).
"""
from dataclasses import dataclass

import torch

from ..native import hip_ops


@dataclass
class QuantizedTensor:
    data: torch.Tensor      # int8 (int4: two per byte)
    scales: torch.Tensor    # fp32 [n / group_size]
    zeros: torch.Tensor     # fp32 [n / group_size] (asymmetric) or empty
    shape: torch.Size
    group_size: int
    bits: int
    dtype: torch.dtype

    def dequantize(self):
        return dequantize(self)


def _ref_quantize(x, gs, bits, asym, stochastic=False):
    xf = x.float().reshape(-1, gs)
    if asym:
        mn, mx = xf.min(1, keepdim=True).values, xf.max(1, keepdim=True).values
        scale = (mx - mn) / (2**bits - 1)
        scale = torch.where(scale == 0, torch.ones_like(scale), scale)
        t = (xf - mn) / scale
        t = torch.floor(t + torch.rand_like(t)) if stochastic else torch.round(t)
        q = t.clamp(0, 2**bits - 1)
        zeros = mn.reshape(-1)
    else:
        amax = xf.abs().max(1, keepdim=True).values
        qmax = 2**(bits - 1) - 1
        scale = amax / qmax
        scale = torch.where(scale == 0, torch.ones_like(scale), scale)
        t = xf / scale
        t = torch.floor(t + torch.rand_like(t)) if stochastic else torch.round(t)
        q = t.clamp(-qmax, qmax)
        zeros = torch.empty(0)
    q = q.to(torch.int16).reshape(-1)
    if bits == 4:
        lo = (q[0::2] & 0xF)
        hi = (q[1::2] & 0xF) << 4
        packed = (lo | hi).to(torch.uint8).view(torch.int8)
    else:
        packed = q.to(torch.int8) if not asym else q.to(torch.uint8).view(torch.int8)
    return packed, scale.reshape(-1), zeros


def _ref_dequantize(q, scales, zeros, n, gs, bits, dtype):
    if bits == 4:
        u = q.view(torch.uint8).to(torch.int16)
        lo, hi = u & 0xF, (u >> 4) & 0xF
        vals = torch.stack([lo, hi], 1).reshape(-1)
        if zeros.numel() == 0:
            vals = torch.where(vals > 7, vals - 16, vals)
    else:
        vals = q.view(torch.uint8).to(torch.int16) if zeros.numel() else q.to(torch.int16)
    x = vals.float().reshape(-1, gs) * scales.reshape(-1, 1)
    if zeros.numel():
        x = x + zeros.reshape(-1, 1)
    return x.reshape(-1)[:n].to(dtype)


def quantize(x, group_size=256, bits=8, symmetric=True, stochastic_rounding=False, seed=0):
    flat = x.contiguous().reshape(-1)
    n = flat.numel()
    gs = min(group_size, n)
    assert n % gs == 0, f"numel {n} not divisible by group size {gs}"
    if flat.is_cuda:
        q, s, z = hip_ops().quantize(flat, gs, bits, not symmetric, stochastic_rounding, seed)
    else:
        q, s, z = _ref_quantize(flat, gs, bits, not symmetric, stochastic_rounding)
    return QuantizedTensor(q, s, z, x.shape, gs, bits, x.dtype)


def dequantize(qt: QuantizedTensor, dtype=None):
    dtype = dtype or qt.dtype
    n = 1
    for d in qt.shape:
        n *= d
    if qt.data.is_cuda:
        out = hip_ops().dequantize(qt.data, qt.scales, qt.zeros if qt.zeros.numel() else None, n, qt.group_size,
                                   qt.bits, dtype)
    else:
        out = _ref_dequantize(qt.data, qt.scales, qt.zeros, n, qt.group_size, qt.bits, dtype)
    return out.view(qt.shape)


def dequant_reduce(q, scales, nsrc, group_size, out_scale=1.0, dtype=torch.float32):
    """Sum of `nsrc` int8-quantised copies (qgZ intra-node reduction)."""
    if q.is_cuda:
        return hip_ops().dequant_reduce(q, scales, nsrc, group_size, out_scale, dtype)
    n = q.numel() // nsrc
    acc = torch.zeros(n)
    for k in range(nsrc):
        acc += _ref_dequantize(q[k * n:(k + 1) * n], scales[k * (n // group_size):(k + 1) * (n // group_size)],
                               torch.empty(0), n, group_size, 8, torch.float32)
    return (acc * out_scale).to(dtype)


def fake_quantize(x, group_size=256, bits=8, symmetric=True, stochastic_rounding=False):
    """In-place quantise->dequantise (QAT / MoQ), reference `fake_quantizer.cu`."""
    qt = quantize(x, group_size, bits, symmetric, stochastic_rounding)
    x.copy_(dequantize(qt, x.dtype))
    return x


def ds_quantizer(input, groups=1, bit_num=8, sr=False, asym=False):
    """Reference signature: quantise `input` into `groups` groups in place (fake quant)."""
    gs = input.numel() // groups
    return fake_quantize(input, gs, bit_num, not asym, sr)


# ---- the quantizer extension's function names (reference `csrc/quantization/pt_binding.cpp:270-297`)
def ds_quantize_fp32(vals, groups, bits):
    """In-place symmetric fake quantisation of `vals` in `groups` groups (fp16 / bf16 / fp32 alike here)."""
    return ds_quantizer(vals, groups, bits)


def ds_sr_quantize_fp32(vals, groups, bits):
    return ds_quantizer(vals, groups, bits, sr=True)


def ds_quantize_asym_fp32(vals, groups, bits):
    return ds_quantizer(vals, groups, bits, asym=True)


def ds_sr_quantize_asym_fp32(vals, groups, bits):
    return ds_quantizer(vals, groups, bits, sr=True, asym=True)


ds_quantize_fp16, ds_sr_quantize_fp16 = ds_quantize_fp32, ds_sr_quantize_fp32
ds_quantize_asym_fp16, ds_sr_quantize_asym_fp16 = ds_quantize_asym_fp32, ds_sr_quantize_asym_fp32


def dequantize_int8_to_half_experimental(data, scales_and_zeros, num_group, group_size):
    """Asymmetric int8 codes [num_group * group_size] + [num_group, 2] (scale, minimum) -> fp16."""
    x = data.reshape(num_group, group_size).float()
    sz = scales_and_zeros.reshape(num_group, 2).float()
    return (x * sz[:, :1] + sz[:, 1:]).to(torch.float16).reshape(-1)


def dequantize_int4_to_half_experimental(data, scales_and_zeros, num_group, group_size):
    """Packed asymmetric int4 codes (two per byte, high nibble first) + (scale, minimum) per group -> fp16."""
    b = data.reshape(-1).to(torch.uint8)
    codes = torch.stack([(b >> 4) & 0xF, b & 0xF], dim=1).reshape(-1)
    return dequantize_int8_to_half_experimental(codes, scales_and_zeros, num_group, group_size)


def swizzle_quant(input_vals, groups, num_bits, quant_type=None, pipeline_size=1, nodes=1, devices_per_node=1):
    """Quantise with the destination chunks re-ordered [local index][node] (qgZ first level). Returns (codes,
    scales)."""
    from ...runtime.zero.zeropp import swizzle_quant as _sw
    qt = _sw(input_vals.reshape(-1), nodes, devices_per_node, input_vals.numel() // groups, num_bits)
    return qt.data, qt.scales


def quantized_reduction(input_vals, input_scales, in_groups, out_groups, num_bits, quant_type=None,
                        devices_per_node=1):
    """Dequantise `devices_per_node` stacked copies, sum, re-quantise (qgZ second step). Returns (codes, scales)."""
    from ...runtime.zero.zeropp import quantized_reduction as _qr
    gs = input_vals.numel() // in_groups
    qt = _qr(input_vals.reshape(-1), input_scales.reshape(-1), devices_per_node, gs, num_bits)
    return qt.data, qt.scales

