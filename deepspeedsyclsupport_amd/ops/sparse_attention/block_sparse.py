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
        o_full = o
        if D < 128:
            o = o[..., :D]
        if need_grad:
            ctx.save_for_backward(q, k, v, o_full, lse)
            ctx.layout, ctx.blk, ctx.scale = layout, blk, float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, H, L, D = q.shape
        qtiles, nqt, lay_u8, blk = build_bwd_lut(ctx.layout, ctx.blk, L, H, q.device)
        if D < 128:
            pad = (0, 128 - D)
            q, k, v, do = (torch.nn.functional.pad(t, pad) for t in (q, k, v, do))
        elif do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, ctx.scale, 2, qtiles, nqt, lay_u8, blk)
        if D < 128:
            dq, dk, dv = dq[..., :D], dk[..., :D], dv[..., :D]
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
