"""Block-sparse attention on the gfx950 flash kernel (reference: the Triton SDD / softmax / DSD kernels of
`ops/sparse_attention/{matmul.py:628, softmax.py:224}` driven by `sparse_self_attention.py`).

Forward: `csrc/attn/flash_fwd.hip` in its SPARSE instantiation — every workgroup (one 128-row query block of one
head) visits only the 64-key tiles its layout rows touch, listed in a LUT built here once per (layout, sequence
length), and masks inside a tile at the layout's block granularity. Work and K/V traffic therefore scale with the
layout density. Head dims below 128 are zero-padded to 128 (zeros change neither QK^T nor the kept part of PV).

Backward: `csrc/attn/flash_bwd.hip` in its SPARSE instantiation (reference: the transposed DSD/SDD products of
`matmul.py:605` and the sparse softmax backward `softmax.py:213`) — every workgroup (256 keys of one head) visits
only the 32-row query tiles its key block meets in the layout (a column LUT built here) and masks at the layout's
block granularity, recomputing P from the forward's LSE. No [L, L] tensor is ever built; work scales with density.
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


_BWD_LUTS = {}


def build_bwd_lut(layout, blk, L, H, device):
    """Column LUT of the sparse backward: (qtiles int32 [H, nkb, T] = 32-row query tiles met by each 256-key block,
    ascending, nqt int32 [H, nkb], layout uint8 [LH, nb, nb] at granularity blk' = min(blk, 128), blk')."""
    key = _lut_key(layout, blk, L, device) + (H,)
    hit = _BWD_LUTS.get(key)
    if hit is not None:
        return hit
    lay = layout.to(torch.bool)
    if lay.shape[0] > 1 and bool((lay == lay[:1]).all()):
        lay = lay[:1]
    if blk > 128:  # the kernel masks at <= 128-row granularity: refine the layout
        f = blk // 128
        lay = lay.repeat_interleave(f, 1).repeat_interleave(f, 2)
        blk = 128
    LH, nb, _ = lay.shape
    g = 16
    fine = lay.repeat_interleave(blk // g, 1).repeat_interleave(blk // g, 2)[:, :L // g, :L // g]
    nkb = (L + 255) // 256
    ntq = L // 32
    fine = torch.nn.functional.pad(fine, (0, nkb * 16 - fine.shape[2]))
    met = fine.reshape(LH, ntq, 2, nkb, 16).any(4).any(2)      # [LH, ntq, nkb]
    met = met.permute(0, 2, 1).contiguous()                     # [LH, nkb, ntq]
    nqt = met.sum(-1).to(torch.int32)
    T = max(int(nqt.max()), 1)
    order = torch.sort((~met).to(torch.int8), dim=-1, stable=True).indices[..., :T].to(torch.int32)
    if LH == 1 and H > 1:
        order, nqt = order.expand(H, nkb, T), nqt.expand(H, nkb)
    out = (order.contiguous().to(device), nqt.contiguous().to(device), lay.to(torch.uint8).contiguous().to(device),
           blk)
    if len(_BWD_LUTS) > 64:
        _BWD_LUTS.clear()
    _BWD_LUTS[key] = out
    return out


def token_bias(layout, blk, L, H, dtype, device):
    """Additive [1, H, L, L] bias: 0 where the layout allows, -inf elsewhere. Reference semantics for tests and
    host fallbacks only — the kernels never build it."""
    lay = layout.to(torch.bool)
    tok = lay.repeat_interleave(blk, 1).repeat_interleave(blk, 2)[:, :L, :L].to(device)
    if tok.shape[0] == 1 and H > 1:
        tok = tok.expand(H, L, L)
    return torch.zeros((1, H, L, L), dtype=dtype, device=device).masked_fill_(~tok[None], float("-inf"))


class BlockSparseAttnFn(torch.autograd.Function):
    """q/k/v bf16 [B, H, L, D], L a multiple of 128; kbias [B, L] / abias [L, L] / rpe [H or 1, L, L] are optional
    fp32 additive biases on the scaled scores, applied inside the kernels (no gradient flows to them, as in the
    reference's sparse softmax)."""

    @staticmethod
    def forward(ctx, q, k, v, layout, blk, scale, kbias, abias, rpe):
        B, H, L, D = q.shape
        tiles, ntiles, lay_u8, qorder = build_lut(layout, blk, L, q.device)
        if D < 128:
            pad = (0, 128 - D)
            qp, kp, vp = (torch.nn.functional.pad(t, pad) for t in (q, k, v))
        else:
            qp, kp, vp = q, k, v
        need_grad = any(t.requires_grad for t in (q, k, v))
        o, lse = hip_ops().flash_fwd_sparse(qp, kp, vp, float(scale), tiles, ntiles, qorder, lay_u8, int(blk),
                                              need_grad, kbias, abias, rpe)
        o_full = o
        if D < 128:
            o = o[..., :D]
        if need_grad:
            ctx.save_for_backward(q, k, v, o_full, lse, *[t for t in (kbias, abias, rpe) if t is not None])
            ctx.has_bias = (kbias is not None, abias is not None, rpe is not None)
            ctx.layout, ctx.blk, ctx.scale = layout, blk, float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, *bias = ctx.saved_tensors
        it = iter(bias)
        kbias, abias, rpe = (next(it) if has else None for has in ctx.has_bias)
        B, H, L, D = q.shape
        qtiles, nqt, lay_u8, blk = build_bwd_lut(ctx.layout, ctx.blk, L, H, q.device)
        if D < 128:
            pad = (0, 128 - D)
            q, k, v, do = (torch.nn.functional.pad(t, pad) for t in (q, k, v, do))
        elif do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, ctx.scale, 2, qtiles, nqt, lay_u8, blk, kbias, abias, rpe)
        if D < 128:
            dq, dk, dv = dq[..., :D], dk[..., :D], dv[..., :D]
        return dq, dk, dv, None, None, None, None, None, None


def native_ok(q, k, v, blk):
    """Can the gfx950 block-sparse kernels take these tensors? (16-bit device tensors, same shapes, head dim <= 128;
    fp16 runs in bf16; sequence lengths that are not a multiple of 128 are padded with masked keys)"""
    B, H, L, D = q.shape
    return (q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and k.dtype == q.dtype and v.dtype == q.dtype
            and k.shape == q.shape and v.shape == q.shape and D <= 128 and D % 8 == 0 and L % blk == 0
            and blk in (16, 32, 64, 128, 256))


def _additive(mask, mode, shape_tail):
    """Mask in 'add' mode is added as is; in 'mul' mode 0 drops (-inf) and anything else keeps (0)."""
    m = mask.to(torch.float32)
    if mode == "mul":
        m = torch.where(m != 0, torch.zeros_like(m), torch.full_like(m, float("-inf")))
    return m.reshape(*shape_tail)


def block_sparse_attention(q, k, v, layout, blk, scale=None, key_padding_mask=None, attn_mask=None, rpe=None,
                           key_padding_mask_mode="add", attn_mask_mode="mul"):
    """q/k/v [B, H, L, D] bf16 (fp16 accepted: computed in bf16), layout [H or 1, L/blk, L/blk] ->
    softmax(QK^T*scale + rpe + key_padding_mask + attn_mask, masked by layout) V. The masks and the relative
    position embedding are applied inside the kernels (reference `ops/sparse_attention/softmax.py:37-157`); no
    [B, H, L, L] tensor is built. L only needs to be a multiple of the block size: it is padded to a multiple of 128
    with keys masked out through the per-key bias."""
    B, H, L, D = q.shape
    scale = D**-0.5 if scale is None else scale
    out_dtype = q.dtype
    if q.dtype != torch.bfloat16:
        q, k, v = q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)
    kb = _additive(key_padding_mask, key_padding_mask_mode, (B, L)) if key_padding_mask is not None else None
    ab = _additive(attn_mask, attn_mask_mode, (L, L)) if attn_mask is not None else None
    rp = rpe.to(torch.float32).reshape(-1, L, L) if rpe is not None else None
    Lp = -(-L // 128) * 128
    if Lp != L:
        padn = Lp - L
        q, k, v = (torch.nn.functional.pad(t, (0, 0, 0, padn)) for t in (q, k, v))
        kb = torch.nn.functional.pad(kb if kb is not None else q.new_zeros((B, L), dtype=torch.float32), (0, padn),
                                     value=float("-inf"))
        if ab is not None:
            ab = torch.nn.functional.pad(ab, (0, padn, 0, padn))
        if rp is not None:
            rp = torch.nn.functional.pad(rp, (0, padn, 0, padn))
        nb = layout.shape[1]
        nbp = -(-Lp // blk)
        if nbp > nb:  # padded query rows / keys get their own diagonal blocks (the keys are masked by kbias)
            lay = torch.zeros(layout.shape[0], nbp, nbp, dtype=layout.dtype)
            lay[:, :nb, :nb] = layout
            for i in range(nb, nbp):
                lay[:, i, i] = 1
            layout = lay
    kb, ab, rp = (None if t is None else t.contiguous() for t in (kb, ab, rp))
    out = BlockSparseAttnFn.apply(q, k, v, layout, blk, scale, kb, ab, rp)
    if Lp != L:
        out = out[:, :, :L]
    return out if out.dtype == out_dtype else out.to(out_dtype)
