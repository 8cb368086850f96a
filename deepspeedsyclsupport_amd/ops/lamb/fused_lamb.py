"""FusedLamb (reference `deepspeed/ops/lamb/fused_lamb.py`): per-parameter LAMB with trust-ratio clamping.

Device params use the 2-pass `lamb_flat` kernel (moments + norm partials, then trust-ratio update).
"""
import torch

from .. import reference
from ..native import hip_ops


class FusedLamb(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False,
                 weight_decay=0.0, max_grad_norm=0.0, max_coeff=10.0, min_coeff=0.01, amsgrad=False):
        if amsgrad:
            raise RuntimeError("FusedLamb does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm, max_coeff=max_coeff, min_coeff=min_coeff)
        super().__init__(params, defaults)
        self.lamb_coeffs = []

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.lamb_coeffs = []
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                s = st["step"]
                bc1 = 1 - beta1**s if group["bias_correction"] else 1.0
                bc2 = 1 - beta2**s if group["bias_correction"] else 1.0
                if p.is_cuda:
                    c = hip_ops().lamb_flat(p.data.view(-1), st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1),
                                            p.grad.contiguous().view(-1), None, group["lr"], beta1, beta2,
                                            group["eps"], group["weight_decay"], bc1, bc2, 1.0, group["max_coeff"],
                                            group["min_coeff"])
                    self.lamb_coeffs.append(c)
                else:
                    self.lamb_coeffs.append(
                        reference.lamb_update(p.data, st["exp_avg"], st["exp_avg_sq"], p.grad, group["lr"], beta1,
                                              beta2, group["eps"], group["weight_decay"], s, group["bias_correction"],
                                              1.0, group["max_coeff"], group["min_coeff"]))
        return loss

    def get_lamb_coeffs(self):
        return [float(c) for c in self.lamb_coeffs]
