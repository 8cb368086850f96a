"""Block-sparse attention on the gfx950 flash kernel (reference: the Triton SDD / softmax / DSD kernels of
`ops/sparse_attention/{matmul.py:628, softmax.py:224}` driven by `sparse_self_attention.py`).

Forward: `csrc/attn/flash_fwd.hip` in its SPARSE instantiation — every workgroup (one 128-row query block of one
head) visits only the 64-key tiles its layout rows touch, listed in a LUT built here once per (layout, sequence
length), and masks inside a tile at the layout's block granularity. Work and K/V traffic therefore scale with the
layout density. Head dims below 128 are zero-padded to 128 (zeros change neither QK^T nor the kept part of PV).

Backward: the memory-efficient attention backward fed with our (O, LSE) and the layout as an additive -inf bias,
the same interchange the dense training path uses (`ops/attention.py`). It is exact for the sparse forward; its
work is dense in the sequence length.
"""
import torch

from ..native import hip_ops

_LUTS = {}


def _lut_key(layout, blk, L, device):
    import hashlib
    digest = hashlib.sha1(layout.detach().to("cpu", torch.uint8).contiguous().numpy().tobytes()).hexdigest()
    return (digest, tuple(layout.shape), blk, L, str(device))


def build_lut(layout, blk, L, device):
    """layout [H, nb, nb] (0/1) -> (tiles int32 [LH, nqb, T], ntiles int32 [LH, nqb], layout uint8 [LH, nb, nb],
    qorder int32 [LH, nqb] = query blocks by descending tile count, the kernel's launch order).

    LH = 1 when every head shares one layout. Tile t of query block qb is listed when any key of 64-key tile t is
    allowed for any of the 128 query rows of qb; the tile lists are ascending."""
    key = _lut_key(layout, blk, L, device)
    hit = _LUTS.get(key)
    if hit is not None:
        return hit
    lay = layout.to(torch.bool)
    if lay.shape[0] > 1 and bool((lay == lay[:1]).all()):
        lay = lay[:1]
    LH, nb, _ = lay.shape
    assert nb * blk >= L and L % 128 == 0 and L % blk == 0
    g = min(blk, 64)                                             # common fine grid
    fine = lay.repeat_interleave(blk // g, 1).repeat_interleave(blk // g, 2)[:, :L // g, :L // g]
    q128 = fine.reshape(LH, L // 128, 128 // g, L // g).any(2) if g < 128 else fine
    t64 = q128.reshape(LH, L // 128, L // 64, 64 // g).any(-1)  # [LH, nqb, ntile]
    ntiles = t64.sum(-1).to(torch.int32)
    T = max(int(ntiles.max()), 1)
    order = torch.sort((~t64).to(torch.int8), dim=-1, stable=True).indices[..., :T].to(torch.int32)
    qorder = torch.sort(ntiles, dim=-1, descending=True, stable=True).indices.to(torch.int32)  # heaviest first
    lut = (order.contiguous().to(device), ntiles.contiguous().to(device),
           lay.to(torch.uint8).contiguous().to(device), qorder.contiguous().to(device))
    if len(_LUTS) > 64:
        _LUTS.clear()
    _LUTS[key] = lut
    return lut


def token_bias(layout, blk, L, H, dtype, device):
    """Additive [1, H, L, L] bias: 0 where the layout allows, -inf elsewhere (backward of the sparse forward)."""
    lay = layout.to(torch.bool)
    tok = lay.repeat_interleave(blk, 1).repeat_interleave(blk, 2)[:, :L, :L].to(device)
    if tok.shape[0] == 1 and H > 1:
        tok = tok.expand(H, L, L)
    return torch.zeros((1, H, L, L), dtype=dtype, device=device).masked_fill_(~tok[None], float("-inf"))


class BlockSparseAttnFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, layout, blk, scale):
        B, H, L, D = q.shape
        tiles, ntiles, lay_u8, qorder = build_lut(layout, blk, L, q.device)
        if D < 128:
            pad = (0, 128 - D)
            qp, kp, vp = (torch.nn.functional.pad(t, pad) for t in (q, k, v))
        else:
            qp, kp, vp = q, k, v
        need_grad = any(t.requires_grad for t in (q, k, v))
        o, lse = hip_ops().flash_fwd_sparse(qp, kp, vp, float(scale), tiles, ntiles, qorder, lay_u8, int(blk),
                                              need_grad)
        if D < 128:
            # keep the [B, L, H, D] memory layout the kernel wrote: the efficient-attention backward reads O with
            # that layout (a [B, H, L, D]-contiguous O gives wrong dK/dV and can fault — tools/probe_sparse_bwd.py)
            o_bl = torch.empty((B, L, H, D), dtype=o.dtype, device=o.device).transpose(1, 2)
            o_bl.copy_(o[..., :D])
            o = o_bl
        if need_grad:
            ctx.save_for_backward(q, k, v, o, lse)
            ctx.layout, ctx.blk, ctx.scale = layout, blk, float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, H, L, D = q.shape
        bias = token_bias(ctx.layout, ctx.blk, L, H, q.dtype, q.device).expand(B, H, L, L)
        z = torch.zeros((), dtype=torch.int64, device=q.device)
        do = do if do.stride(-1) == 1 else do.contiguous()
        dq, dk, dv, _ = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
            do, q, k, v, bias, o, lse, z, z, 0.0, [True, True, True, False], False, scale=ctx.scale)
        return dq, dk, dv, None, None, None


def native_ok(q, k, v, blk, rpe=None, key_padding_mask=None, attn_mask=None):
    B, H, L, D = q.shape
    return (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == q.dtype and v.dtype == q.dtype
            and k.shape == q.shape and v.shape == q.shape and D <= 128 and D % 8 == 0 and L % 128 == 0
            and L % blk == 0 and blk in (16, 32, 64, 128, 256) and rpe is None and key_padding_mask is None
            and attn_mask is None and all(t.stride(-1) == 1 and all(x % 8 == 0 for x in t.stride()[:3])
                                          for t in (q, k, v)))


def block_sparse_attention(q, k, v, layout, blk, scale=None):
    """q/k/v [B, H, L, D] bf16, layout [H or 1, L/blk, L/blk] -> softmax(QK^T*scale masked by layout) V."""
    scale = q.shape[-1]**-0.5 if scale is None else scale
    return BlockSparseAttnFn.apply(q, k, v, layout, blk, scale)
