"""Weight-only int8 linear layers for decode: group-quantised weights stored once in MFMA operand order.

Reference counterparts (behaviour): the weight-only int8 inference path of `transformer_inference`
(`csrc/transformer/inference/csrc/pt_binding.cpp` `ds_vector_matmul_int8` + `dequantize.cu:15-86`) and v2's
`mixed_gemm` (CUTLASS). Both dequantise (or stream-dequantise) a row-major weight into a library GEMM.

MI355X design (`csrc/gemv/skinny_int8.hip`): a decode GEMM is a weight stream, and the HBM stream only runs at full
rate when each 16-byte-per-lane load covers long contiguous segments — which the MFMA operand layout read from a
row-major matrix does not (measured 4.4-5 TB/s loads-only). Inference weights are constants, so the int8 matrix is
re-laid ONCE at quantisation time:

    qsh[nb, kq, lane, :] = q[16 nb + (lane % 16), 64 kq + 16 (lane // 16) : +16]     (int8, 1 KB per 16 x 64 tile)
    ssh[nb, group, r]    = scales[16 nb + r, group]

so one contiguous 1 KB load per wave is exactly the B operand of two v_mfma_f32_16x16x32_bf16. Prefill (more than 16
token rows) dequantises straight from the shuffled layout into a row-major bf16 temporary (`dequant_sh`) for the
library GEMM.
"""
import torch
import torch.nn.functional as F

from .native import hip_ops
from .quantizer import QuantizedTensor, dequantize, quantize

MAX_DECODE_ROWS = 16


class PendingAcc:
    """A decode GEMV whose fp32 sums still sit in the stream's split-K workspace (no bias applied yet). Exactly one
    of the `finalize*` methods must run before the next weight-only GEMV on the stream: each converts the sums,
    fuses the element-wise op that consumes the projection anyway, and re-zeroes the workspace — one kernel instead
    of finalize + consumer (`csrc/gemv/skinny_finalize.hip`)."""

    def __init__(self, acc, lead_shape, N, bias=None):
        self.acc, self.lead, self.N, self.bias = acc, tuple(lead_shape), N, bias
        self.M = 1
        for d in self.lead:
            self.M *= d
        self.done = False

    def _take(self):
        if self.done:
            raise RuntimeError("the workspace of this GEMV was already consumed")
        self.done = True
        return self.acc

    def finalize(self):
        return hip_ops().skinny_finalize(self._take(), self.M, self.N, self.bias).view(*self.lead, self.N)

    def finalize_rms(self, residual, weight, eps):
        """-> (RMSNorm(sums + bias + residual) * weight, sums + bias + residual)"""
        r = None if residual is None else residual.reshape(self.M, self.N).contiguous()
        y, res = hip_ops().skinny_finalize_rms(self._take(), self.M, self.N, self.bias, r, weight, eps)
        return y.view(*self.lead, self.N), res.view(*self.lead, self.N)

    def finalize_gated(self, act_code):
        """-> act(gate + b) * (up + b) for a fused [gate | up] projection"""
        return hip_ops().skinny_finalize_gated(self._take(), self.M, self.N, self.bias, act_code).view(
            *self.lead, self.N // 2)


def raw_ok(x, bias=None):
    return x.is_cuda and x.dtype == torch.bfloat16 and x.numel() // x.shape[-1] <= MAX_DECODE_ROWS and \
        (bias is None or bias.dtype == torch.bfloat16)


def preshuffle(q, scales, group_size):
    """Row-major int8 q [N, K] + fp32 scales [N * K / gs] -> (qsh [NB, K/64, 64, 16], ssh [NB, K/gs, 16]), N padded
    to NB * 16 rows with zero weights / zero scales."""
    N, K = q.shape
    if K % 64 or group_size % 64 or K % group_size:
        raise ValueError(f"preshuffle needs K and group size multiples of 64 (K={K}, gs={group_size})")
    nb = (N + 15) // 16
    s = scales.reshape(N, K // group_size)
    if nb * 16 != N:
        q = F.pad(q, (0, 0, 0, nb * 16 - N))
        s = F.pad(s, (0, 0, 0, nb * 16 - N))
    qsh = q.reshape(nb, 16, K // 64, 4, 16).permute(0, 2, 3, 1, 4).reshape(nb, K // 64, 64, 16).contiguous()
    ssh = s.reshape(nb, 16, K // group_size).permute(0, 2, 1).contiguous()
    return qsh, ssh


def unshuffle(qsh, ssh, N):
    """Inverse of `preshuffle`: (q [N, K] int8, scales [N * K / gs] fp32)."""
    nb, kq = qsh.shape[0], qsh.shape[1]
    q = qsh.reshape(nb, kq, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(nb * 16, kq * 64)[:N]
    s = ssh.permute(0, 2, 1).reshape(nb * 16, ssh.shape[1])[:N]
    return q.contiguous(), s.reshape(-1).contiguous()


class Int8Weight:
    """Symmetric group-quantised weight [N, K] kept in the pre-shuffled layout."""

    def __init__(self, w, group_size=64):
        N, K = w.shape
        self.shape = w.shape
        self.dtype = w.dtype
        self.group_size = min(group_size, K)
        qt = quantize(w.contiguous(), group_size=self.group_size, bits=8, symmetric=True)
        self.qsh, self.ssh = preshuffle(qt.data.view(N, K), qt.scales, self.group_size)

    @staticmethod
    def supported(w, bits=8, group_size=64):
        return bits == 8 and w.dim() == 2 and w.shape[1] % 64 == 0 and min(group_size, w.shape[1]) % 64 == 0 \
            and w.shape[1] % min(group_size, w.shape[1]) == 0

    def nbytes(self):
        return self.qsh.numel() + self.ssh.numel() * 4

    def materialize(self, dtype=None):
        dtype = dtype or self.dtype
        if self.qsh.is_cuda and dtype == torch.bfloat16:
            return hip_ops().dequant_sh(self.qsh, self.ssh, self.shape[0], self.group_size)
        q, s = unshuffle(self.qsh, self.ssh, self.shape[0])
        qt = QuantizedTensor(q.reshape(-1), s, torch.empty(0, device=q.device), self.shape, self.group_size, 8,
                             self.dtype)
        return dequantize(qt, dtype)

    def raw(self, x, bias=None):
        """Decode GEMV without its finalize pass (see `PendingAcc`); `raw_ok(x, bias)` must hold."""
        K = x.shape[-1]
        acc = hip_ops().skinny_q_raw(x.reshape(-1, K).contiguous(), self.qsh, self.ssh, self.shape[0],
                                     self.group_size, 8)
        return PendingAcc(acc, x.shape[:-1], self.shape[0], bias)

    def linear(self, x, bias=None):
        """x [..., K] -> x . W^T (+ bias). Up to 16 token rows on a GPU: the fused MFMA stream (no bf16 weight is
        ever written); otherwise dequantise + library GEMM."""
        K = x.shape[-1]
        M = x.numel() // K
        if x.is_cuda and x.dtype == torch.bfloat16 and M <= MAX_DECODE_ROWS and \
                (bias is None or bias.dtype == torch.bfloat16):
            y = hip_ops().skinny_i8_sh(x.reshape(M, K).contiguous(), self.qsh, self.ssh, bias, self.shape[0],
                                       self.group_size)
            return y.view(*x.shape[:-1], self.shape[0])
        return F.linear(x, self.materialize(x.dtype), bias)
