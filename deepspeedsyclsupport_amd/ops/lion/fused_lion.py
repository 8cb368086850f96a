"""FusedLion (reference `deepspeed/ops/lion/fused_lion.py`)."""
import torch

from .. import reference
from ..native import hip_ops


def lion_flat_update(p, m, g, lr, beta1, beta2, weight_decay, grad_scale=1.0, lp=None):
    if p.is_cuda:
        hip_ops().lion_flat(p, m, g, lp, lr, beta1, beta2, weight_decay, grad_scale)
    else:
        reference.lion_update(p, m, g, lr, beta1, beta2, weight_decay, grad_scale, lp)


class FusedLion(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), weight_decay=0.0, set_grad_none=True):
        super().__init__(params, dict(lr=lr, betas=betas, weight_decay=weight_decay))
        self.set_grad_none = set_grad_none

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                st["step"] += 1
                lion_flat_update(p.data.view(-1), st["exp_avg"].view(-1), p.grad.contiguous().view(-1), group["lr"],
                                 b1, b2, group["weight_decay"])
        return loss
