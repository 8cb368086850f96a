"""bf16 linear layers for decode: the weight stored once in MFMA operand order (`csrc/gemv/skinny_bf16_sh.hip`).

Reference counterpart (behaviour): the bf16 / fp16 decode GEMMs of `transformer_inference` (`qkv_gemm`,
`vector_matmul`, `mlp_gemm`, `csrc/transformer/inference/csrc/pt_binding.cpp`) on the row-major weight.

A decode GEMM is a weight stream; read from a row-major matrix the MFMA operand layout is 16 rows x 64 B per load
instruction, which holds the stream at 3 - 4.2 TB/s. Inference weights are constants, so — as for the int8 / int4
streams (`ops/int8_gemv.py`) — the matrix is re-laid ONCE:

    wsh[nb, kq, h, lane, :] = w[16 nb + (lane % 16), 64 kq + 16 (lane // 16) + 8 h : +8]      (2 KB per 16 x 64 tile)

and every 16-byte-per-lane load reads 1 KB contiguous. With more than 16 token rows (prefill) the library GEMM runs
on a row-major matrix: the copy kept next to the shuffled one when `keep_row_major` (twice the weight memory, sized
for 288 GB of HBM), else a temporary un-shuffled right before the GEMM.
"""
import torch
import torch.nn.functional as F

from .int8_gemv import MAX_DECODE_ROWS, PendingAcc, raw_ok  # noqa: F401
from .native import hip_ops


def preshuffle16(w):
    """Row-major bf16 w [N, K] -> wsh [NB, K/64, 2, 64, 8], N padded to NB * 16 rows with zeros."""
    N, K = w.shape
    if K % 64:
        raise ValueError(f"preshuffle16 needs K a multiple of 64 (K={K})")
    nb = (N + 15) // 16
    if nb * 16 != N:
        w = F.pad(w, (0, 0, 0, nb * 16 - N))
    # [nb, r, kq, g, h, j] -> [nb, kq, h, g, r, j]  (lane = 16 g + r)
    return w.reshape(nb, 16, K // 64, 4, 2, 8).permute(0, 2, 4, 3, 1, 5).reshape(nb, K // 64, 2, 64, 8).contiguous()


def unshuffle16(wsh, N):
    """Inverse of `preshuffle16` (any device, PyTorch ops)."""
    nb, kq = wsh.shape[0], wsh.shape[1]
    return wsh.reshape(nb, kq, 2, 4, 16, 8).permute(0, 4, 1, 3, 2, 5).reshape(nb * 16, kq * 64)[:N].contiguous()


class Bf16Weight:
    """A bf16 weight [N, K] kept in the pre-shuffled decode layout (and, optionally, row-major for prefill)."""

    def __init__(self, w, keep_row_major=False):
        self.shape = w.shape
        self.dtype = w.dtype
        self.wsh = preshuffle16(w)
        self.row_major = w.contiguous() if keep_row_major else None

    @staticmethod
    def supported(w):
        return w.dim() == 2 and w.dtype == torch.bfloat16 and w.shape[1] % 64 == 0

    def nbytes(self):
        return (self.wsh.numel() + (0 if self.row_major is None else self.row_major.numel())) * 2

    def materialize(self, dtype=None):
        if self.row_major is not None:
            w = self.row_major
        elif self.wsh.is_cuda:
            w = hip_ops().unshuffle_sh16(self.wsh, self.shape[0])
        else:
            w = unshuffle16(self.wsh, self.shape[0])
        return w if dtype in (None, w.dtype) else w.to(dtype)

    def raw(self, x, bias=None):
        """Decode GEMV without its finalize pass (see `PendingAcc`); `raw_ok(x, bias)` must hold."""
        K = x.shape[-1]
        acc = hip_ops().skinny_b16_raw(x.reshape(-1, K).contiguous(), self.wsh, self.shape[0])
        return PendingAcc(acc, x.shape[:-1], self.shape[0], bias)

    def linear(self, x, bias=None):
        K = x.shape[-1]
        M = x.numel() // K
        if raw_ok(x, bias):
            return hip_ops().skinny_b16_sh(x.reshape(M, K).contiguous(), self.wsh, bias, self.shape[0]).view(
                *x.shape[:-1], self.shape[0])
        return F.linear(x, self.materialize(x.dtype), bias)
