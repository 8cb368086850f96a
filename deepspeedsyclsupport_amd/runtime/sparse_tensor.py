"""Sparse (row-sparse) gradient tensors for embeddings (reference `runtime/sparse_tensor.py`, engine sparse
all-reduce `engine.py:2447-2518`): an embedding gradient touched by few tokens travels as (indices, rows) and is
all-gathered instead of all-reducing the dense [vocab, hidden] matrix."""
import torch

from .. import comm as dist


class SparseTensor:

    def __init__(self, dense_tensor=None):
        self.orig_dense_tensor = dense_tensor
        self.is_sparse = dense_tensor is not None and dense_tensor.is_sparse
        if dense_tensor is not None:
            if dense_tensor.is_sparse:
                dense_tensor = dense_tensor.coalesce()
                self.indices = dense_tensor.indices().flatten()
                self.values = dense_tensor.values()
            else:
                rows = dense_tensor.abs().sum(dim=1).nonzero().flatten()
                self.indices = rows
                self.values = dense_tensor[rows]
            self.dense_size = list(dense_tensor.size())
        else:
            self.indices = self.values = self.dense_size = None

    def to_coo_tensor(self):
        return torch.sparse_coo_tensor(self.indices.unsqueeze(0), self.values, self.dense_size)

    @staticmethod
    def type():
        return "deepspeed.SparseTensor"

    def to_dense(self):
        out = torch.zeros(self.dense_size, dtype=self.values.dtype, device=self.values.device)
        out.index_add_(0, self.indices, self.values)
        return out

    def sparse_size(self):
        return self.indices.numel() + self.values.numel(), self.dense_size[0] * self.dense_size[1]

    def add(self, b):
        self.indices = torch.cat([self.indices, b.indices])
        self.values = torch.cat([self.values, b.values])

    def __str__(self):
        ss, ds = self.sparse_size()
        return f"DeepSpeed.SparseTensor(indices_size={self.indices.size()}, values_size={self.values.size()}, " \
               f"dense_size={self.dense_size}, reduction_factor={ds / max(ss, 1)})"

    __repr__ = __str__


def sparse_allreduce(sparse: SparseTensor, group=None, average=True):
    """All-gather variable-length (indices, rows) from every rank and sum (reference engine.sparse_allreduce)."""
    world = dist.get_world_size(group)
    n = torch.tensor([sparse.indices.numel()], device=sparse.indices.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    mx = int(max(int(s) for s in sizes))
    pad_i = torch.zeros(mx, dtype=sparse.indices.dtype, device=sparse.indices.device)
    pad_v = torch.zeros((mx, ) + tuple(sparse.values.shape[1:]), dtype=sparse.values.dtype,
                        device=sparse.values.device)
    pad_i[:n.item()] = sparse.indices
    pad_v[:n.item()] = sparse.values
    all_i = [torch.empty_like(pad_i) for _ in range(world)]
    all_v = [torch.empty_like(pad_v) for _ in range(world)]
    dist.all_gather(all_i, pad_i, group=group)
    dist.all_gather(all_v, pad_v, group=group)
    sparse.indices = torch.cat([i[:int(s)] for i, s in zip(all_i, sizes)])
    sparse.values = torch.cat([v[:int(s)] for v, s in zip(all_v, sizes)])
    if average:
        sparse.values = sparse.values / world
    return sparse
