"""Weight-only mixed-precision GEMMs of inference v2 (reference `inference/v2/kernels/cutlass_ops/mixed_gemm/
mixed_gemm.py` `MixedGEMM` and `moe_gemm/{moe_gemm,mixed_moe_gemm}.py` `MoEGEMM` / `MixedMoEGEMM`, built by
`InferenceCutlassBuilder`). Same call contracts — `kernel(output, hidden_states, weights, scales, biases)` with
weights [in, out] quantised per output channel (int8, or int4 packed two per byte along `out`), `act(x W + b)`
written into `output` — on the MI355X int8 kernels instead of CUTLASS:

 * int8: the per-channel weight is re-laid ONCE (cached per weight tensor) into the pre-shuffled MFMA operand layout
   of `csrc/gemv/skinny_int8.hip`; up to 16 token rows run the fused-dequant MFMA stream, larger batches dequantise
   straight from that layout (`dequant_sh`) into the library GEMM;
 * int4: re-packed ONCE into the operand layout of `csrc/gemv/skinny_int4.hip` (K a multiple of 128): decode streams
   half a byte per weight through the fused-dequant MFMA kernel, larger batches dequantise from that layout
   (`dequant_sh4`) into the library GEMM;
 * MoE: per-expert weights [E, in, out] with expert-sorted token counts, each expert one of the above (or plain
   bf16 when unquantised) — the grouped-GEMM kernels of `ops/moe_ops.py` cover the unquantised MoE path.
"""
import torch
import torch.nn.functional as F

from .int4_gemv import Int4Weight
from .int8_gemv import Int8Weight, preshuffle
from .transformer.functional import ACT_CODES
from . import reference

_ACTS = {"gelu": "gelu", "silu": "silu", "relu": "relu", "identity": "identity", None: "identity"}


def _act_name(act):
    name = getattr(act, "name", act)
    name = str(name).lower() if name is not None else None
    if name not in _ACTS:
        raise ValueError(f"unsupported activation {act}")
    return _ACTS[name]


def unpack_int4(packed):
    """[in, out // 2] uint8 (low nibble = even column, two's-complement nibbles) -> int8 [in, out]."""
    lo = (packed & 0x0F).to(torch.int16)
    hi = (packed >> 4).to(torch.int16)
    lo = torch.where(lo > 7, lo - 16, lo)
    hi = torch.where(hi > 7, hi - 16, hi)
    return torch.stack([lo, hi], dim=-1).reshape(packed.shape[0], -1).to(torch.int8)


def pack_int4(q):
    """Inverse of `unpack_int4` for int8 values in [-8, 7]."""
    u = (q.to(torch.int16) & 0x0F).to(torch.uint8).reshape(q.shape[0], -1, 2)
    return (u[..., 0] | (u[..., 1] << 4)).contiguous()


class _PerChannel(Int8Weight):
    """An already-quantised per-output-channel weight in the pre-shuffled layout (one scale group spans K)."""

    def __init__(self, q_in_out, scales, dtype):
        K, N = q_in_out.shape
        self.shape = torch.Size([N, K])
        self.dtype = dtype
        self.group_size = K
        self.qsh, self.ssh = preshuffle(q_in_out.t().contiguous(), scales.float().reshape(-1).contiguous(), K)


class MixedGEMM:
    """act(hidden_states @ dequant(weights) + biases) -> output, weights [in, out] int8 / packed int4."""

    def __init__(self, fp_dtype=torch.bfloat16, act_fn="identity", num_bits=8):
        if num_bits not in (4, 8):
            raise ValueError(f"unsupported num_bits {num_bits}: 4 or 8")
        if fp_dtype not in (torch.float16, torch.bfloat16):
            raise ValueError(f"unsupported dtype {fp_dtype}")
        self.fp_dtype, self.num_bits, self.act = fp_dtype, num_bits, _act_name(act_fn)
        self._cache = {}

    def _weight(self, weights, scales):
        key = (weights.data_ptr(), scales.data_ptr(), tuple(weights.shape))
        w = self._cache.get(key)
        if w is None:
            q = unpack_int4(weights) if self.num_bits == 4 else weights
            if self.num_bits == 4 and q.shape[0] % 128 == 0:
                # per-output-channel scales = one scale group spanning K
                K, N = q.shape
                w = Int4Weight(q=q.t().contiguous(), scales=scales.float().reshape(-1).contiguous(), group_size=K,
                               dtype=self.fp_dtype)
            elif q.shape[0] % 64 == 0:
                w = _PerChannel(q, scales, self.fp_dtype)
            else:  # K not a multiple of 64: keep the dequantised weight (no pre-shuffled layout possible)
                w = (q.float() * scales.float().reshape(1, -1)).t().contiguous().to(self.fp_dtype)
            self._cache[key] = w
        return w

    def __call__(self, output, hidden_states, weights, scales, biases=None):
        w = self._weight(weights, scales)
        x = hidden_states.to(self.fp_dtype)
        b = biases.to(self.fp_dtype) if biases is not None else None
        y = w.linear(x, b) if isinstance(w, (Int8Weight, Int4Weight)) else F.linear(x, w, b)
        if self.act != "identity":
            y = reference.ACTS[ACT_CODES[self.act]](y.float()).to(y.dtype)
        output.copy_(y.reshape(output.shape))
        return output


class MoEGEMM:
    """Per-expert GEMMs over expert-sorted tokens: output[rows of e] = act(hidden[rows of e] @ W_e + b_e).
    weights [E, in, out] (fp) or quantised with `num_bits` and scales [E, out]; total_rows_before_expert [E] int64
    (inclusive prefix sums of the per-expert token counts, reference contract)."""

    def __init__(self, fp_dtype=torch.bfloat16, act_fn="identity", num_bits=None):
        self.fp_dtype, self.act, self.num_bits = fp_dtype, _act_name(act_fn), num_bits
        self._mixed = MixedGEMM(fp_dtype, "identity", num_bits) if num_bits else None

    def __call__(self, output, hidden_states, weights, total_rows_before_expert, biases=None, scales=None):
        ends = total_rows_before_expert.tolist()
        start = 0
        for e, end in enumerate(ends):
            if end > start:
                x = hidden_states[start:end]
                b = biases[e] if biases is not None else None
                if self._mixed is not None:
                    y = torch.empty(end - start, output.shape[-1], dtype=self.fp_dtype, device=output.device)
                    self._mixed(y, x, weights[e], scales[e], b)
                else:
                    y = F.linear(x.to(self.fp_dtype), weights[e].t().to(self.fp_dtype), b)
                if self.act != "identity":
                    y = reference.ACTS[ACT_CODES[self.act]](y.float()).to(y.dtype)
                output[start:end].copy_(y)
            start = end
        return output


MixedMoEGEMM = MoEGEMM


def mixed_gemm(output, hidden_states, weights, scales, biases=None, num_bits=8, act_fn="identity"):
    return MixedGEMM(output.dtype, act_fn, num_bits)(output, hidden_states, weights, scales, biases)


def moe_gemm(output, hidden_states, weights, total_rows_before_expert, biases=None, act_fn="identity"):
    return MoEGEMM(output.dtype, act_fn)(output, hidden_states, weights, total_rows_before_expert, biases)
