"""Block-sparse matrix products as a standalone op (reference `ops/sparse_attention/matmul.py:628` `MatMul`, Triton
SDD / DSD / DDS kernels).

`layout` [H, rows / block, cols / block] marks the non-zero blocks; a sparse operand is stored as
[batch, nnz, block, block] with blocks in `layout.nonzero()` order.
  * "sdd": dense x dense -> sparse (only the marked output blocks are computed);
  * "dsd": sparse x dense -> dense;
  * "dds": dense x sparse -> dense.
Every mode gathers the operand blocks it needs and issues ONE batched GEMM over the non-zero blocks (the library's
batched MFMA GEMM), then scatters / accumulates with an index-add: work and traffic are O(nnz), and the whole op is
differentiable. The fused attention path (`sparse_self_attention.py` on the SPARSE flash kernels) never materialises
these intermediates; this op exists for code written against the three-step MatMul / Softmax / MatMul API.
"""
import torch


class MatMul:

    def __init__(self, layout, block, mode, trans_a=False, trans_b=False, bench=False):
        if mode not in ("sdd", "dsd", "dds"):
            raise NotImplementedError("Supported modes are: sdd, dsd, dds")
        self.layout = layout.long()
        self.block, self.mode, self.trans_a, self.trans_b = block, mode, trans_a, trans_b
        nz = self.layout.nonzero()
        self.h, self.i, self.j = nz[:, 0], nz[:, 1], nz[:, 2]
        self.nnz = nz.shape[0]
        self.spdims = tuple(self.layout.shape)

    def _idx(self, device):
        return self.h.to(device), self.i.to(device), self.j.to(device)

    def __call__(self, a, b):
        blk = self.block
        H, R, C = self.spdims
        if self.mode == "sdd":
            a = a.transpose(-1, -2) if self.trans_a else a       # [B, H, M, K]
            b = b.transpose(-1, -2) if self.trans_b else b       # [B, H, K, N]
            h, i, j = self._idx(a.device)
            B_, _, M, K = a.shape
            N = b.shape[-1]
            ab = a.reshape(B_, H, M // blk, blk, K)[:, h, i]                    # [B, nnz, blk, K]
            bb = b.reshape(B_, H, K, N // blk, blk).permute(0, 1, 3, 2, 4)[:, h, j]   # [B, nnz, K, blk]
            return torch.matmul(ab, bb)
        if self.mode == "dsd":
            h, i, j = self._idx(b.device)
            if self.trans_a:       # the stored blocks are those of A^T: block (i, j) of A^T is block (j, i) of A
                a, i, j = a.transpose(-1, -2), j, i
                R = self.spdims[2]
            b = b.transpose(-1, -2) if self.trans_b else b       # [B, H, K, N]
            B_, _, K, N = b.shape
            rows = b.reshape(B_, H, K // blk, blk, N)[:, h, j]                  # [B, nnz, blk, N]
            prod = torch.matmul(a, rows)                                        # [B, nnz, blk, N]
            out = torch.zeros(B_, H * R, blk, N, dtype=prod.dtype, device=prod.device)
            out = out.index_add(1, h * R + i, prod)
            return out.view(B_, H, R * blk, N)
        # dds
        h, i, j = self._idx(a.device)
        if self.trans_b:
            b, i, j = b.transpose(-1, -2), j, i
            C = self.spdims[1]
        a = a.transpose(-1, -2) if self.trans_a else a           # [B, H, M, K]
        B_, _, M, K = a.shape
        cols = a.reshape(B_, H, M, K // blk, blk).permute(0, 1, 3, 2, 4)[:, h, i]   # [B, nnz, M, blk]
        prod = torch.matmul(cols, b)                                            # [B, nnz, M, blk]
        out = torch.zeros(B_, H * C, M, blk, dtype=prod.dtype, device=prod.device)
        out = out.index_add(1, h * C + j, prod)
        return out.view(B_, H, C, M, blk).permute(0, 1, 3, 2, 4).reshape(B_, H, M, C * blk)
