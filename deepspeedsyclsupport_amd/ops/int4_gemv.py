"""Weight-only int4 linear layers: group-quantised weights packed once in MFMA operand order.

Reference counterparts (behaviour): inference v2's CUTLASS `mixed_gemm` with `num_bits=4`
(`inference/v2/kernels/cutlass_ops/mixed_gemm/mixed_gemm.py`; built by `op_builder/inference_cutlass_builder.py`) and
the int4 mode of the v1 weight quantiser (`runtime/weight_quantizer.py`).

MI355X design (`csrc/gemv/skinny_int4.hip`): symmetric int4 q in [-8, 7] is stored as the nibble u = q + 8, eight per
32-bit word, in the order the decode kernel's MFMA wants its B operand:

    word i of q4[nb, kq, lane] = W[16 nb + (lane % 16), 128 kq + 32 i + 8 (lane // 16) + j],  j = 0..7,
                                 weight j in nibble (j / 2 if j is even else 4 + j // 2)
    s4[nb, group, r]           = scales[16 nb + r, group]

A wave-wide load is 1 KB contiguous; `0x4300 | u` is the bf16 number 128 + u, so the kernel builds operand elements with
one and-or per register and corrects the offset with sum(x). Decode (<= 16 token rows) streams the packed weight
(0.5 byte + scales per parameter); prefill dequantises from the same layout (`dequant_sh4`) into a bf16 temporary for
the library GEMM.
"""
import torch
import torch.nn.functional as F

from .int8_gemv import PendingAcc
from .native import hip_ops
from .quantizer import quantize

MAX_DECODE_ROWS = 16
_NIBBLE_OF = (0, 4, 1, 5, 2, 6, 3, 7)  # operand element j -> nibble position inside its word


def group_ok(K, group_size):
    gs = min(group_size, K)
    return K % 128 == 0 and K % gs == 0 and (gs in (32, 64) or gs % 128 == 0)


def unpack_pairs(packed):
    """The quantiser's int4 output (two two's-complement nibbles per byte, low nibble first) -> int8 values."""
    u = packed.view(torch.uint8).to(torch.int16)
    v = torch.stack([u & 0xF, (u >> 4) & 0xF], -1).reshape(-1)
    return torch.where(v > 7, v - 16, v).to(torch.int8)


def pack_int4_operands(q, scales, group_size):
    """Row-major int8 q [N, K] with values in [-8, 7] + fp32 scales [N * K / gs] -> (q4 int8 bytes
    [NB, K/128, 64, 16], s4 fp32 [NB, K/gs, 16]); N padded to NB * 16 rows of zero weights and zero scales."""
    N, K = q.shape
    if not group_ok(K, group_size):
        raise ValueError(f"int4 packing needs K % 128 == 0 and a group size of 32, 64 or a multiple of 128 "
                         f"(K={K}, gs={group_size})")
    nb = (N + 15) // 16
    s = scales.reshape(N, K // group_size)
    if nb * 16 != N:
        q = F.pad(q, (0, 0, 0, nb * 16 - N))
        s = F.pad(s, (0, 0, 0, nb * 16 - N))
    u = (q.to(torch.int32) + 8) & 0xF                                    # [NB*16, K]
    u = u.reshape(nb, 16, K // 128, 4, 4, 8).permute(0, 2, 4, 1, 3, 5)   # [nb, kq, g, r, i, j]
    shifts = torch.tensor([4 * n for n in _NIBBLE_OF], dtype=torch.int32, device=q.device)
    words = (u << shifts).sum(-1, dtype=torch.int64)                     # nibbles are disjoint: sum == or
    words = torch.where(words >= 2**31, words - 2**32, words).to(torch.int32)
    q4 = words.reshape(nb, K // 128, 64, 4).contiguous().view(torch.int8).reshape(nb, K // 128, 64, 16)
    s4 = s.reshape(nb, 16, K // group_size).permute(0, 2, 1).contiguous().float()
    return q4, s4


def unpack_int4_operands(q4, s4, N):
    """Inverse of `pack_int4_operands`: (q [N, K] int8 in [-8, 7], scales [N * K / gs] fp32)."""
    nb, kq = q4.shape[0], q4.shape[1]
    words = q4.contiguous().view(torch.int32).reshape(nb, kq, 4, 16, 4).to(torch.int64) & 0xFFFFFFFF  # [nb,kq,g,r,i]
    shifts = torch.tensor([4 * n for n in _NIBBLE_OF], dtype=torch.int64, device=q4.device)
    u = (words.unsqueeze(-1) >> shifts) & 0xF                            # [nb, kq, g, r, i, j]
    q = (u - 8).permute(0, 3, 1, 4, 2, 5).reshape(nb * 16, kq * 128)[:N].to(torch.int8)
    s = s4.permute(0, 2, 1).reshape(nb * 16, s4.shape[1])[:N]
    return q.contiguous(), s.reshape(-1).contiguous()


class Int4Weight:
    """Symmetric group-quantised int4 weight [N, K] kept in the packed operand layout."""

    def __init__(self, w=None, group_size=128, q=None, scales=None, dtype=None):
        """Quantise `w`, or adopt an already quantised (q int8 [N, K] in [-8, 7], scales [N * K / gs]) pair."""
        if w is not None:
            N, K = w.shape
            self.shape, self.dtype = w.shape, w.dtype
            self.group_size = min(group_size, K)
            qt = quantize(w.contiguous(), group_size=self.group_size, bits=4, symmetric=True)
            q, scales = unpack_pairs(qt.data).view(N, K), qt.scales
        else:
            self.shape, self.dtype = q.shape, dtype or torch.bfloat16
            self.group_size = min(group_size, q.shape[1])
        self.q4, self.s4 = pack_int4_operands(q, scales.float(), self.group_size)

    @staticmethod
    def supported(w, bits=4, group_size=128):
        return bits == 4 and w.dim() == 2 and group_ok(w.shape[1], group_size)

    def nbytes(self):
        return self.q4.numel() + self.s4.numel() * 4

    def materialize(self, dtype=None):
        dtype = dtype or self.dtype
        if self.q4.is_cuda:
            w = hip_ops().dequant_sh4(self.q4, self.s4, self.shape[0], self.group_size)
            return w if dtype == torch.bfloat16 else w.to(dtype)
        q, s = unpack_int4_operands(self.q4, self.s4, self.shape[0])
        K = self.shape[1]
        return (q.float().reshape(self.shape[0], K // self.group_size, self.group_size) *
                s.reshape(self.shape[0], -1, 1)).reshape(self.shape[0], K).to(dtype)

    def raw(self, x, bias=None):
        """Decode GEMV without its finalize pass (see `int8_gemv.PendingAcc`); `int8_gemv.raw_ok` must hold."""
        K = x.shape[-1]
        acc = hip_ops().skinny_q_raw(x.reshape(-1, K).contiguous(), self.q4, self.s4, self.shape[0], self.group_size,
                                     4)
        return PendingAcc(acc, x.shape[:-1], self.shape[0], bias)

    def linear(self, x, bias=None):
        """x [..., K] -> x . W^T (+ bias). Up to 16 token rows on a GPU: the fused MFMA stream over the packed weight;
        otherwise dequantise + library GEMM."""
        K = x.shape[-1]
        M = x.numel() // K
        if x.is_cuda and x.dtype == torch.bfloat16 and M <= MAX_DECODE_ROWS and \
                (bias is None or bias.dtype == torch.bfloat16):
            y = hip_ops().skinny_i4(x.reshape(M, K).contiguous(), self.q4, self.s4, bias, self.shape[0],
                                    self.group_size)
            return y.view(*x.shape[:-1], self.shape[0])
        return F.linear(x, self.materialize(x.dtype), bias)
