"""PLD, eigenvalue, sparse tensors (reference `tests/unit/runtime/test_pld.py`, `sparse_tensor/*`)."""
import math

import torch

from ..common import run_distributed


def test_pld_schedule():
    from deepspeedsyclsupport_amd.runtime.progressive_layer_drop import ProgressiveLayerDrop
    p = ProgressiveLayerDrop(theta=0.5, gamma=0.01)
    assert p.get_theta() == 1.0
    p.update_state(100)
    assert math.isclose(p.get_theta(), 0.5 * math.exp(-1.0) + 0.5)
    assert p.get_state()["progressive_layer_drop"] is True


def test_eigenvalue_quadratic():
    from deepspeedsyclsupport_amd.runtime.eigenvalue import Eigenvalue

    class Quad(torch.nn.Module):

        def __init__(self):
            super().__init__()
            self.layers = torch.nn.ModuleList([torch.nn.Linear(4, 1, bias=False) for _ in range(2)])

        def forward(self, x):
            # loss = 0.5 * c_i * ||w_i||^2 -> Hessian eigenvalue c_i
            return 0.5 * 3.0 * self.layers[0].weight.pow(2).sum() + 0.5 * 6.0 * self.layers[1].weight.pow(2).sum()

    m = Quad()
    ev = Eigenvalue(max_iter=50, tol=1e-6, layer_name="layers", layer_num=2)
    vals = ev.compute_eigenvalue(m, loss=m(None))
    assert abs(vals[0] - 0.5) < 1e-3 and abs(vals[1] - 1.0) < 1e-3


def _sparse(out):
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.sparse_tensor import SparseTensor, sparse_allreduce
    r = dist.get_rank()
    dense = torch.zeros(10, 3)
    dense[r * 3] = r + 1.0
    dense[9] = 1.0
    st = sparse_allreduce(SparseTensor(dense))
    full = dense.clone()
    dist.all_reduce(full)
    if r == 0:
        torch.save({"got": st.to_dense(), "ref": full / 2}, out)


def test_sparse_allreduce(tmp_path):
    out = str(tmp_path / "s.pt")
    run_distributed(_sparse, 2, out)
    d = torch.load(out, weights_only=True)
    torch.testing.assert_close(d["got"], d["ref"])


def test_partition_balanced_and_norms():
    from deepspeedsyclsupport_amd.runtime.utils import (clip_grad_norm_, get_global_norm_of_tensors,
                                                        partition_balanced, partition_uniform)
    assert partition_uniform(10, 3) == [0, 4, 7, 10]
    parts = partition_balanced([1, 1, 1, 10, 1, 1, 1, 1], 3)
    sizes = [sum([1, 1, 1, 10, 1, 1, 1, 1][a:b]) for a, b in zip(parts, parts[1:])]
    assert parts[0] == 0 and parts[-1] == 8 and max(sizes) == 10
    ps = [torch.nn.Parameter(torch.ones(4)) for _ in range(2)]
    for p in ps:
        p.grad = torch.full((4, ), 3.0)
    n = clip_grad_norm_(ps, 1.0)
    assert abs(n - math.sqrt(8 * 9)) < 1e-5
    assert abs(get_global_norm_of_tensors([p.grad for p in ps]) - 1.0) < 1e-4
