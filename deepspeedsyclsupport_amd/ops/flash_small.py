"""Small-head flash attention with additive biases and attention dropout (`csrc/attn/flash_small.hip`).

Serves the two reference paths that need more than plain causal attention:
 * DS4Science Evoformer attention (`ops/deepspeed4science/evoformer_attn.py:14-106`): softmax(QK^T/sqrt(D) + bias1 +
   bias2) V over [B, N, S, H, D] with a per-key mask bias [B, N, 1, 1, S] and a pair bias [B, 1, H, S, S] shared by
   the N MSA rows; gradients for Q, K, V and both biases;
 * the BERT training layer (`ops/transformer/transformer.py` + `csrc/transformer/softmax_kernels.cu`,
   `dropout_kernels.cu`): additive per-key attention mask and attention-probability dropout.

Tensors are [Z, S, H, D] views (any z/s/h strides, unit last stride): Z folds the batch dims, bias1 is [Z, S] and
bias2 [Z / b2_div, H, S, S]. No [Z, H, S, S] tensor is ever materialised — not the bias sum, not P, not the dropout
mask (regenerated in the backward from a Philox-4x32-7 stream keyed by (seed, z, h, query, key)).
"""
import weakref

import numpy as np
import torch

SUPPORTED_D = (32, 64)


def supported(q, *, need_dtype=True):
    """True when the native kernel handles q's shape / dtype / device ([..., S, H, D] views, unit last stride)."""
    return (q.is_cuda and q.shape[-1] in SUPPORTED_D and (not need_dtype or q.dtype in (torch.bfloat16, torch.float16))
            and q.stride(-1) == 1)


def _fix(t):
    """The kernel reads 16-B chunks: unit last stride, (z, s, h) strides in multiples of 8 elements, 16-B base."""
    if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:3]) or t.data_ptr() % 16:
        return t.contiguous()
    return t


def new_seed():
    """Per-call dropout seed from torch's default (CPU) generator, so `torch.manual_seed` makes runs repeatable."""
    return int(torch.randint(0, 2**62, (1, )).item())


class FlashSmallFunc(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, b1, b2, b2_div, scale, pdrop, seed):
        from .native import hip_ops
        if q.shape[1] != k.shape[1] and any(ctx.needs_input_grad[:5]):
            raise NotImplementedError("flash_small: the backward needs the same query and key length")
        q, k, v = _fix(q), _fix(k), _fix(v)
        o, lse = hip_ops().flash_small_fwd(q, k, v, b1, b2, int(b2_div), float(scale), float(pdrop), int(seed))
        ctx.save_for_backward(q, k, v, o, lse, b1, b2)
        ctx.cfg = (int(b2_div), float(scale), float(pdrop), int(seed))
        ctx.want = (b1 is not None and ctx.needs_input_grad[3], b2 is not None and ctx.needs_input_grad[4])
        return o

    @staticmethod
    def backward(ctx, do):
        from .native import hip_ops
        q, k, v, o, lse, b1, b2 = ctx.saved_tensors
        b2_div, scale, pdrop, seed = ctx.cfg
        dq, dk, dv, db1, db2 = hip_ops().flash_small_bwd(_fix(do), q, k, v, o, lse, b1, b2, b2_div, scale, pdrop,
                                                         seed, ctx.want[0], ctx.want[1])
        db1 = db1.to(b1.dtype) if ctx.want[0] else None
        db2 = db2.to(b2.dtype) if ctx.want[1] else None
        return dq, dk, dv, db1, db2, None, None, None, None


def flash_small(q, k, v, bias1=None, bias2=None, b2_div=1, scale=None, dropout_p=0.0, seed=None):
    """q [Z, S, H, D], k/v [Z, Sk, H, D] -> o [Z, S, H, D] (contiguous). bias1 [Z, Sk], bias2 [Z / b2_div, H, S, Sk]
    (q dtype). Sk != S (cross-attention) is forward-only."""
    scale = q.shape[-1]**-0.5 if scale is None else scale
    if dropout_p > 0.0 and seed is None:
        seed = new_seed()
    if bias2 is not None and not bias2.is_contiguous():
        bias2 = bias2.contiguous()
    if bias1 is not None and bias1.stride(-1) != 1:
        bias1 = bias1.contiguous()
    return FlashSmallFunc.apply(q, k, v, bias1, bias2, b2_div, scale, dropout_p, seed or 0)


_CAUSAL_BIAS = {}
BIAS2_MAX_BYTES = 64 << 20  # a per-(query, key) mask is expanded over heads for the kernel: only while that stays small


def _causal_bias(H, S, dtype, device):
    key = (H, S, dtype, str(device))
    if key not in _CAUSAL_BIAS:
        m = torch.full((S, S), torch.finfo(dtype).min, dtype=dtype, device=device).triu_(1)
        _CAUSAL_BIAS[key] = m.expand(1, H, S, S).contiguous()
    return _CAUSAL_BIAS[key]


_PER_KEY = {}  # id(mask) -> (weakref to it, its version counter, verdict)


def _is_per_key(m):
    """Is the 4-D mask constant over heads and queries? Broadcast dims and stride-0 (expanded) dims say so for free;
    a dense [B, 1|H, Nq, Nk] mask (what HF's SDPA mask helpers build from a padding mask) is compared with its first
    row once per tensor object: the verdict is remembered while that object lives, so the layers of an encoder that
    all receive the same mask share one check. Inside a stream capture no host decision may depend on device data:
    the mask then travels as the pair bias, which is always valid."""
    if (m.shape[1] == 1 or m.stride(1) == 0) and (m.shape[2] == 1 or m.stride(2) == 0):
        return True
    if m.is_cuda and torch.cuda.is_current_stream_capturing():
        return False
    hit = _PER_KEY.get(id(m))
    if hit is not None and hit[0]() is m and hit[1] == m._version:
        return hit[2]
    verdict = bool(torch.equal(m, m[:, :1, :1, :].expand_as(m)))
    if len(_PER_KEY) > 256:
        _PER_KEY.clear()
    _PER_KEY[id(m)] = (weakref.ref(m), m._version, verdict)
    return verdict


def attend(q, k, v, mask=None, scale=None, causal=False):
    """Inference attention for encoder / diffusion blocks on the small-head kernel: q [B, Nq, H, D], k/v [B, Nk, H, D]
    (views are fine) -> [B, Nq, H, D], or None when the kernel does not serve the case (the caller keeps its
    library path). `mask` is what HF / diffusers modules hand around: boolean (True = attend) or additive, shaped
    [B, Nk], [B, 1|Nq, Nk] or [B|1, 1|H, 1|Nq, Nk]. A mask that is constant over queries and heads (padding masks,
    also when they arrive expanded) travels as the per-key bias; anything else as the per-(query, key) bias, shared
    over the batch when its batch dim is 1. `causal` adds the triangular bias (CLIP text tower)."""
    B, Nq, H, D = q.shape
    Nk = k.shape[1]
    if not supported(q) or k.dtype != q.dtype or v.dtype != q.dtype or torch.is_grad_enabled() and Nq != Nk:
        return None
    b1 = b2 = None
    b2_div = 1
    if mask is not None:
        m = mask
        if m.dim() == 2:
            m = m[:, None, None, :]
        elif m.dim() == 3:
            m = m[:, None]
        if m.dim() != 4 or m.shape[-1] != Nk or m.shape[0] not in (1, B) or m.shape[1] not in (1, H) \
                or m.shape[2] not in (1, Nq):
            return None
        per_key = _is_per_key(m)
        if per_key:
            m = m[:, :1, :1, :]
        elif m.shape[0] * H * Nq * Nk * q.element_size() > BIAS2_MAX_BYTES:
            return None
        if m.dtype == torch.bool:
            m = torch.zeros(m.shape, dtype=q.dtype, device=q.device).masked_fill_(~m, torch.finfo(q.dtype).min)
        else:
            m = m.to(q.dtype)
        if per_key:
            b1 = m[:, 0, 0, :].expand(B, Nk).contiguous()
        else:
            b2 = m.expand(m.shape[0], H, Nq, Nk).contiguous()
            b2_div = B // m.shape[0]
    if causal:
        if Nq != Nk:
            return None
        cb = _causal_bias(H, Nq, q.dtype, q.device)
        if b2 is None:
            b2, b2_div = cb, B
        else:
            b2 = b2 + cb  # (min + min saturates to -inf in bf16/fp16: still a masked key)
    return flash_small(q, k, v, bias1=b1, bias2=b2, b2_div=b2_div, scale=scale)


# ---------------------------------------------------------------------------------------------- host references
_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def keep_mask(seed, Z, H, S, p):
    """The kernel's dropout keep mask [Z, H, S, S] (bool), recomputed on the host (numpy Philox-4x32-7): one Philox
    call per (z, h, query, 4-key group); output word i decides key 4*group + i (keep iff word >= p * 2^32)."""
    thresh = np.uint64(min(4294967295, int(p * 4294967296.0)))
    m32 = np.uint64(0xFFFFFFFF)
    row = (np.arange(Z * H * S, dtype=np.uint64))[:, None]
    grp = np.arange((S + 3) // 4, dtype=np.uint64)[None, :]
    c0 = np.broadcast_to(grp, (Z * H * S, grp.shape[1])).copy()
    c1 = np.broadcast_to(row & m32, c0.shape).copy()
    c2 = np.broadcast_to(row >> np.uint64(32), c0.shape).copy()
    c3 = np.full(c0.shape, 0x5bd1e995, dtype=np.uint64)
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(7):
        p0 = np.uint64(_M0) * c0
        p1 = np.uint64(_M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & m32
        hi1, lo1 = p1 >> np.uint64(32), p1 & m32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(_W0)) & m32
        k1 = (k1 + np.uint64(_W1)) & m32
    words = np.stack([c0, c1, c2, c3], axis=-1).reshape(Z * H * S, -1)[:, :S]
    return torch.from_numpy((words >= thresh).reshape(Z, H, S, S))


def reference(q, k, v, bias1=None, bias2=None, b2_div=1, scale=None, keep=None, p=0.0):
    """fp32 PyTorch oracle of the same op (materialises [Z, H, S, S]; for tests)."""
    Z, S, H, D = q.shape
    scale = D**-0.5 if scale is None else scale
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) * scale
    if bias1 is not None:
        s = s + bias1.float()[:, None, None, :]
    if bias2 is not None:
        s = s + bias2.float().repeat_interleave(b2_div, dim=0)
    pr = torch.softmax(s, dim=-1)
    if keep is not None:
        pr = pr * keep.to(pr.device).float() / (1.0 - p)
    return (pr @ vf).permute(0, 2, 1, 3)
