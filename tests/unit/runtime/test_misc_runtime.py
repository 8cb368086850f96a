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
