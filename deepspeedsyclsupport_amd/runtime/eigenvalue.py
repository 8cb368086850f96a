"""Per-layer dominant Hessian eigenvalue by power iteration (reference `runtime/eigenvalue.py:14-160`), used by MoQ
to order layers by sensitivity. Hessian-vector products come from double back-propagation of the layer gradients.
"""
import math

import torch

from ..utils.logging import log_dist


class Eigenvalue:

    def __init__(self, verbose=False, max_iter=100, tol=1e-2, stability=1e-6, gas_boundary_resolution=1,
                 layer_name="", layer_num=0):
        self.verbose = verbose
        self.max_iter = max_iter
        self.tol = tol
        self.stability = stability
        self.gas_boundary_resolution = gas_boundary_resolution
        self.layer_name = layer_name
        self.layer_num = layer_num

    @staticmethod
    def nan_to_num(x):
        return torch.nan_to_num(x, nan=0.0, posinf=0.0, neginf=0.0)

    def normalize(self, v):
        norm = math.sqrt(sum(float((x * x).sum()) for x in v))
        return [x / (norm + self.stability) for x in v]

    @staticmethod
    def inner_product(xs, ys):
        return sum(float((x * y).sum()) for x, y in zip(xs, ys))

    def get_layers(self, module):
        m = module
        for part in self.layer_name.split("."):
            if part:
                m = getattr(m, part)
        return list(m)[:self.layer_num] if self.layer_num else list(m)

    def compute_eigenvalue(self, module, loss=None, device=None, scale=1.0):
        """Dominant |eigenvalue| of the Hessian restricted to each block's parameters. If `loss` is None the params'
        `.grad` must come from a backward with create_graph=True."""
        blocks = self.get_layers(module)
        out = []
        for bi, block in enumerate(blocks):
            params = [p for p in block.parameters() if p.requires_grad]
            if loss is not None:
                grads = torch.autograd.grad(loss, params, create_graph=True, retain_graph=True, allow_unused=True)
            else:
                grads = [p.grad for p in params]
            pairs = [(p, g) for p, g in zip(params, grads) if g is not None and g.requires_grad]
            if not pairs:
                out.append(0.0)
                continue
            params, grads = [p for p, _ in pairs], [g for _, g in pairs]
            v = self.normalize([torch.randn_like(p) for p in params])
            eig, prev = 0.0, None
            for i in range(self.max_iter):
                hv = torch.autograd.grad(grads, params, grad_outputs=v, retain_graph=True)
                hv = [self.nan_to_num(h.float()) for h in hv]
                eig = self.inner_product(hv, v)
                v = self.normalize(hv)
                if prev is not None and abs(eig - prev) / (abs(prev) + self.stability) < self.tol:
                    break
                prev = eig
            out.append(abs(eig) / scale)
            if self.verbose:
                log_dist(f"block {bi}: eigenvalue {out[-1]:.4e} after {i + 1} iterations", ranks=[0])
        return self.post_process(out)

    @staticmethod
    def post_process(values):
        """Normalise to (0, 1] by the max; a block with no curvature signal stays 0 here (the per-parameter map
        below gives it the neutral 1.0, as the reference's `post_process` does)."""
        mx = max(values) if values else 0.0
        return [v / mx if mx > 0 else 0.0 for v in values]

    def compute_block_eigenvalue(self, module, loss=None, device=None, scale=1.0):
        """{id(param): (normalised eigenvalue, block index)} — the form MoQ consumes (reference
        `runtime/eigenvalue.py:67-143` returns the same map)."""
        values = self.compute_eigenvalue(module, loss=loss, device=device, scale=scale)
        out = {}
        for i, (block, v) in enumerate(zip(self.get_layers(module), values)):
            for p in block.parameters():
                out[id(p)] = (v if v != 0.0 else 1.0, i)
        return out
