"""Block-sparse softmax as a standalone op (reference `ops/sparse_attention/softmax.py:224` `Softmax`).

Input and output are sparse [batch, nnz, block, block] in `layout.nonzero()` order. A row of the attention matrix is
spread over the non-zero blocks of its block row, so the row maximum and the row sum are segment reductions over
those blocks (`scatter_reduce`), everything else is elementwise: O(nnz) work, differentiable. Scale, relative
position bias, key padding mask and attention mask are applied per block before the softmax, exactly the operands the
fused kernel path takes.
"""
import torch


class Softmax:

    def __init__(self, layout, block, bench=False):
        self.layout = layout.long()
        self.block = block
        nz = self.layout.nonzero()
        self.h, self.i, self.j = nz[:, 0], nz[:, 1], nz[:, 2]
        self.spdims = tuple(self.layout.shape)

    def _blocks_of(self, dense, device):
        """[.., H or 1, M, N] (broadcastable) -> its blocks at the non-zero positions [.., nnz, blk, blk]."""
        blk = self.block
        H, R, C = self.spdims
        d = dense.to(device)
        while d.dim() < 4:
            d = d.unsqueeze(0)
        d = d.expand(d.shape[0], H, R * blk, C * blk)
        return d.reshape(d.shape[0], H, R, blk, C, blk).permute(0, 1, 2, 4, 3, 5)[:, self.h.to(device),
                                                                                   self.i.to(device),
                                                                                   self.j.to(device)]

    def __call__(self, x, scale=1.0, rpe=None, key_padding_mask=None, attn_mask=None, key_padding_mask_mode="add",
                 attn_mask_mode="add"):
        for mode in (key_padding_mask_mode, attn_mask_mode):
            if mode not in ("add", "mul"):
                raise ValueError('mask modes are "add" (a float bias) or "mul" (0 = masked out)')
        blk = self.block
        H, R, C = self.spdims
        dev = x.device
        h, i, j = self.h.to(dev), self.i.to(dev), self.j.to(dev)
        s = x.float() * scale
        if rpe is not None:
            s = s + self._blocks_of(rpe.float(), dev)
        if key_padding_mask is not None:        # [B, N]
            kp = key_padding_mask.to(dev).float().view(key_padding_mask.shape[0], C, blk)[:, j]     # [B, nnz, blk]
            if key_padding_mask_mode == "mul":
                kp = torch.where(kp == 0, torch.full_like(kp, float("-inf")), torch.zeros_like(kp))
            s = s + kp[:, :, None, :]
        if attn_mask is not None:               # [M, N]
            am = self._blocks_of(attn_mask.float(), dev)
            if attn_mask_mode == "mul":
                am = torch.where(am == 0, torch.full_like(am, float("-inf")), torch.zeros_like(am))
            s = s + am
        B_ = s.shape[0]
        seg = (h * R + i).view(1, -1, 1).expand(B_, -1, blk)                     # segment of every (block, row)
        row_max = torch.full((B_, H * R, blk), float("-inf"), device=dev)
        row_max = row_max.scatter_reduce(1, seg, s.amax(-1), "amax", include_self=True)
        row_max = torch.where(torch.isinf(row_max), torch.zeros_like(row_max), row_max)   # fully masked rows
        e = torch.exp(s - row_max.gather(1, seg)[..., None])
        row_sum = torch.zeros(B_, H * R, blk, device=dev).scatter_add(1, seg, e.sum(-1))
        out = e / row_sum.gather(1, seg)[..., None].clamp_min(1e-30)
        return out.to(x.dtype)
