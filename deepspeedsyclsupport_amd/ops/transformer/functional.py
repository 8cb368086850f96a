"""Autograd wrappers for the fused transformer kernels (training path).

Each op runs the gfx950 kernel for device tensors and the fp32 PyTorch reference for host tensors. Parity: the
fused pieces of the reference training layer (`csrc/transformer/ds_transformer_cuda.cpp:154-300`: LN, bias+GELU,
transform_0213, softmax) and inference kernels (`rms_norm.cu`, `apply_rotary_pos_emb.cu`, `gelu.cu` gated acts).
"""
import torch
import torch.nn.functional as F

from .. import reference
from ..native import hip_ops

ACT_CODES = {"silu": 0, "swiglu": 0, "gelu_tanh": 1, "gelu_new": 1, "gelu_pytorch_tanh": 1, "gelu": 2, "geglu": 2,
             "relu": 3, "reglu": 3, "identity": 4}


# --------------------------------------------------------------------------------------------------- RMSNorm
class _RMSNormFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, w, eps, residual):
        y, res, rstd = hip_ops().rms_fwd(x, residual, w, eps)
        h = res if residual is not None else x
        ctx.save_for_backward(h, w, rstd)
        ctx.has_res = residual is not None
        return (y, res) if ctx.has_res else y

    @staticmethod
    def backward(ctx, dy, dres=None):
        h, w, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        if dres is not None:
            dres = dres.contiguous()
        dx, dw = hip_ops().rms_bwd(dy, h, w, rstd, dres)
        # d(x) == d(residual) when the forward summed them
        return dx, dw, None, (dx if ctx.has_res else None)


_NORM_BWD_MAX_H = 8192    # norm kernels: forward up to 16384 wide rows, backward up to 8192


def _norm_kernel_ok(x, *params):
    if not x.is_cuda or x.shape[-1] % 8:
        return False
    if x.shape[-1] <= _NORM_BWD_MAX_H:
        return True
    needs_grad = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (x, ) + params)
    return x.shape[-1] <= 16384 and not needs_grad


def rms_norm(x, weight, eps=1e-6, residual=None):
    """y = RMSNorm(x [+ residual]) * weight. With `residual`, returns (y, x + residual)."""
    if _norm_kernel_ok(x, weight, residual):
        x = x.contiguous()
        if residual is not None:
            residual = residual.contiguous()
        return _RMSNormFn.apply(x, weight, eps, residual)
    h = x + residual if residual is not None else x
    y = (h.float() * torch.rsqrt(h.float().pow(2).mean(-1, keepdim=True) + eps) * weight.float()).to(x.dtype)
    return (y, h) if residual is not None else y


# --------------------------------------------------------------------------------------------------- LayerNorm
class _LayerNormFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, g, b, eps, residual):
        y, res, mean, rstd = hip_ops().ln_fwd(x, residual, g, b, eps)
        h = res if residual is not None else x
        ctx.save_for_backward(h, g, mean, rstd)
        ctx.has_res = residual is not None
        return (y, res) if ctx.has_res else y

    @staticmethod
    def backward(ctx, dy, dres=None):
        h, g, mean, rstd = ctx.saved_tensors
        dx, dg, db = hip_ops().ln_bwd(dy.contiguous(), h, g, mean, rstd,
                                      dres.contiguous() if dres is not None else None)
        return dx, dg, db, None, (dx if ctx.has_res else None)


def layer_norm(x, weight, bias, eps=1e-5, residual=None):
    if _norm_kernel_ok(x, weight, bias, residual):
        x = x.contiguous()
        if residual is not None:
            residual = residual.contiguous()
        return _LayerNormFn.apply(x, weight, bias, eps, residual)
    h = x + residual if residual is not None else x
    y = torch.nn.functional.layer_norm(h, (h.shape[-1], ), weight, bias, eps)
    return (y, h) if residual is not None else y


# --------------------------------------------------------------------------------------------------- gated act
class _GatedActFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, gu, act):
        ctx.act = act
        ctx.save_for_backward(gu)
        return hip_ops().gated_act_fwd(gu, act)

    @staticmethod
    def backward(ctx, dout):
        (gu, ) = ctx.saved_tensors
        return hip_ops().gated_act_bwd(dout.contiguous(), gu, ctx.act), None


class _GatedActKMajorFn(torch.autograd.Function):
    """Gated activation of a long token batch in training: the kernels also write the token-contiguous ("K-major")
    copies that the neighbouring linears' weight-gradient GEMMs contract over — the output's for the consumer
    (handed over as `out._ds_kmajor`), the input gradient's for the producer (`dgu._ds_kmajor`) — instead of leaving
    them to a separate transpose pass (see `ops/linear.py`)."""

    @staticmethod
    def forward(ctx, gu, act):
        ctx.act = act
        ctx.save_for_backward(gu)
        out, out_t = hip_ops().gated_act_fwd_t(gu, act, 256)
        ctx.mark_non_differentiable(out_t)
        return out, out_t

    @staticmethod
    def backward(ctx, dout, _unused=None):
        (gu, ) = ctx.saved_tensors
        dgu, dgu_t = hip_ops().gated_act_bwd_t(dout.contiguous(), gu, ctx.act, 256)
        dgu._ds_kmajor = dgu_t
        return dgu, None


def gated_activation(gate_up, act="silu"):
    """[.., 2I] = [gate | up] -> act(gate) * up  (SwiGLU for act='silu', GEGLU for 'gelu')."""
    code = ACT_CODES[act]
    if gate_up.is_cuda and (gate_up.shape[-1] // 2) % 8 == 0:
        from ..linear import kmajor_wanted
        rows = gate_up.numel() // gate_up.shape[-1]
        if gate_up.requires_grad and torch.is_grad_enabled() and kmajor_wanted(rows, gate_up.dtype):
            out, out_t = _GatedActKMajorFn.apply(gate_up.contiguous(), code)
            out._ds_kmajor = out_t
            return out
        return _GatedActFn.apply(gate_up.contiguous(), code)
    g, u = gate_up.chunk(2, dim=-1)
    return reference.ACTS[code](g) * u


class _BiasActFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, bias, act):
        ctx.act = act
        ctx.save_for_backward(x, bias)
        return hip_ops().bias_act_fwd(x, bias, act)

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        dx = hip_ops().bias_act_bwd(dy.contiguous(), x, bias, ctx.act)
        db = dx.reshape(-1, dx.shape[-1]).sum(0) if bias is not None else None
        return dx, db, None


def bias_activation(x, bias, act="gelu"):
    code = ACT_CODES[act]
    if x.is_cuda and x.shape[-1] % 8 == 0:
        return _BiasActFn.apply(x.contiguous(), bias, code)
    return reference.ACTS[code](x + bias if bias is not None else x)


# --------------------------------------------------------------------------------------------------- dropout
class _DropoutFn(torch.autograd.Function):
    """y = residual + dropout_p(x + bias) in one kernel; the mask is regenerated from (seed, offset) in backward."""

    @staticmethod
    def forward(ctx, x, bias, residual, p, seed):
        (y, ) = hip_ops().dropout_fwd(x, bias, residual, p, seed, 0, False)
        ctx.p, ctx.seed, ctx.has_bias, ctx.has_res = p, seed, bias is not None, residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = hip_ops().dropout_bwd(dy, ctx.p, ctx.seed, 0)
        db = dx.reshape(-1, dx.shape[-1]).sum(0) if ctx.has_bias else None
        return dx, db, (dy if ctx.has_res else None), None, None


def _dropout_seed():
    # drawn from the host generator: reproducible under torch.manual_seed and restored by activation
    # checkpointing's RNG stash, so a recomputed forward reproduces the same mask; no device sync
    return int(torch.randint(0, 2**62, (1, )).item())


def dropout(x, p, training=True, bias=None, residual=None):
    """residual + dropout(x + bias) (reference `csrc/transformer/dropout_kernels.cu` fused variants)."""
    if not training or p == 0.0:
        y = x if bias is None else x + bias
        return y if residual is None else y + residual
    if x.is_cuda and x.shape[-1] % 8 == 0:
        return _DropoutFn.apply(x.contiguous(), bias, None if residual is None else residual.contiguous(), float(p),
                                _dropout_seed())
    y = F.dropout(x if bias is None else x + bias, p, True)
    return y if residual is None else y + residual


# --------------------------------------------------------------------------------------------------- rotary + split
class _QKVRopeFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, hq, hk, rot, offset, token_major=False):
        q, k, v = hip_ops().qkv_rope_fwd(qkv, cos, sin, pos, hq, hk, rot, offset, token_major)
        ctx.save_for_backward(cos, sin, pos)
        ctx.rot, ctx.offset = rot, offset
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin, pos = ctx.saved_tensors
        dqkv = hip_ops().qkv_rope_bwd(dq, dk, dv, cos, sin, pos, ctx.rot, ctx.offset)
        return dqkv, None, None, None, None, None, None, None, None


def qkv_rope_split(qkv, cos, sin, num_heads, num_kv_heads, rotary_dim=None, position_ids=None, pos_offset=0,
                   token_major=False):
    """qkv [B, S, Hq+2Hk, D] -> q [B,Hq,S,D], k [B,Hk,S,D], v [B,Hk,S,D] with rotate_half RoPE on q and k.
    `token_major=True` returns them as views of [B,S,H,D] memory (what the flash-attention path exchanges with its
    backward without transposing copies).

    `cos`/`sin` are fp32 tables [max_pos, rot/2] (see `reference.rope_tables`)."""
    B, S, NH, D = qkv.shape
    rot = rotary_dim or D
    if qkv.is_cuda and D % 8 == 0 and rot % 16 == 0:
        pos = position_ids.to(torch.int32).contiguous() if position_ids is not None else None
        return _QKVRopeFn.apply(qkv.contiguous(), cos, sin, pos, num_heads, num_kv_heads, rot, pos_offset, token_major)
    q, k, v = qkv.split([num_heads, num_kv_heads, num_kv_heads], dim=2)
    p = position_ids if position_ids is not None else torch.arange(pos_offset, pos_offset + S, device=qkv.device)
    q = reference.apply_rope_half(q, cos, sin, p)
    k = reference.apply_rope_half(k, cos, sin, p)
    return q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)


def apply_rotary_pos_emb(x, cos, sin, position_ids=None, pos_offset=0, rotary_dim=None, interleaved=False,
                         inverse=False):
    """In-place RoPE on a [B, S, H, D] view (inference path; both rotate_half and GPT-J interleaved styles)."""
    rot = rotary_dim or x.shape[-1]
    if x.is_cuda:
        pos = position_ids.to(torch.int32).contiguous() if position_ids is not None else None
        hip_ops().rope_inplace(x, cos, sin, pos, rot, pos_offset, interleaved, inverse)
        return x
    B, S = x.shape[:2]
    p = position_ids if position_ids is not None else torch.arange(pos_offset, pos_offset + S)
    s = -sin if inverse else sin
    if interleaved:
        c, sn = cos[p].float()[..., None, :], s[p].float()[..., None, :]
        if c.dim() == 3:
            c, sn = c[None], sn[None]
        x1, x2 = x[..., 0:rot:2].float(), x[..., 1:rot:2].float()
        o1, o2 = x1 * c - x2 * sn, x2 * c + x1 * sn
        x[..., 0:rot:2], x[..., 1:rot:2] = o1.to(x.dtype), o2.to(x.dtype)
        return x
    x.copy_(reference.apply_rope_half(x, cos, s, p))
    return x


# --------------------------------------------------------------------------------------------------- cross entropy
class _XentFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, logits, labels, ignore_index, smoothing, inplace_grad):
        loss, lse = hip_ops().xent_fwd(logits, labels, ignore_index, smoothing)
        ctx.save_for_backward(logits, labels, lse)
        ctx.ignore_index, ctx.smoothing, ctx.inplace = ignore_index, smoothing, inplace_grad
        return loss

    @staticmethod
    def backward(ctx, dloss):
        logits, labels, lse = ctx.saved_tensors
        dlogits = hip_ops().xent_bwd(logits, labels, lse, dloss.contiguous(), 0.0, ctx.inplace, ctx.ignore_index,
                                     ctx.smoothing)
        return dlogits, None, None, None, None


def cross_entropy(logits, labels, ignore_index=-100, label_smoothing=0.0, reduction="mean", inplace_backward=True):
    """Fused softmax-CE over [N, V] logits (bf16/fp32). `inplace_backward` reuses the logits buffer for the grad."""
    if logits.is_cuda:
        logits2 = logits.reshape(-1, logits.shape[-1])
        labels2 = labels.reshape(-1).contiguous()
        per_tok = _XentFn.apply(logits2, labels2, ignore_index, label_smoothing, inplace_backward)
    else:
        per_tok = reference.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), ignore_index,
                                          label_smoothing)
        labels2 = labels.reshape(-1)
    if reduction == "none":
        return per_tok
    if reduction == "sum":
        return per_tok.sum()
    n = (labels2 != ignore_index).sum().clamp(min=1)
    return per_tok.sum() / n
