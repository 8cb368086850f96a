"""FusedAdam: Adam/AdamW on the gfx950 fused kernel (reference `deepspeed/ops/adam/fused_adam.py:18-191`).

Same constructor/step semantics as the reference (per-parameter `state['step']`, `exp_avg`, `exp_avg_sq`,
`adam_w_mode`, `bias_correction`, `set_grad_none`). Device params go through `ds_hip_ops.adam_multi` (pointer
table in kernel arguments, ≤32 tensors per launch); the ZeRO optimizers call `adam_flat_update` on their flat
fp32 partitions, which also writes the bf16/fp16 model copy in the same pass.
"""
import torch

from .. import reference
from ..native import DTYPE_CODE, hip_ops, use_native


def adam_flat_update(p, m, v, g, step, lr, beta1, beta2, eps, weight_decay, bias_correction=True, adamw_mode=True,
                     grad_scale=1.0, lp=None):
    """In-place Adam on flat tensors. `lp` (optional) receives a low-precision copy of the updated params."""
    bc1 = 1 - beta1**step if bias_correction else 1.0
    bc2 = 1 - beta2**step if bias_correction else 1.0
    if use_native(p, m, v, g, lp):
        hip_ops().adam_flat(p, m, v, g, lp, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale, adamw_mode)
    else:
        reference.adam_update(p, m, v, g, lr, beta1, beta2, eps, weight_decay, step, bias_correction, adamw_mode,
                              grad_scale, lp)


class FusedAdam(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        if set_to_none is None:
            set_to_none = self.set_grad_none
        super().zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None, grad_scaler=None):
        if any(p is not None for p in [grads, output_params, scale, grad_norms]):
            raise RuntimeError("FusedAdam has been updated; step() takes no legacy arguments.")
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = group.get("step", 0)
                    state["exp_avg"] = torch.zeros_like(p)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                state["step"] += 1
                key = (p.dtype, p.grad.dtype, state["step"], p.is_cuda)
                buckets.setdefault(key, []).append(p)
            for (pdt, gdt, step, cuda), ps in buckets.items():
                bc1 = 1 - beta1**step if group["bias_correction"] else 1.0
                bc2 = 1 - beta2**step if group["bias_correction"] else 1.0
                if cuda:
                    hip_ops().adam_multi([p.data for p in ps], [self.state[p]["exp_avg"] for p in ps],
                                         [self.state[p]["exp_avg_sq"] for p in ps], [p.grad for p in ps], [],
                                         group["lr"], beta1, beta2, group["eps"], group["weight_decay"], bc1, bc2,
                                         1.0, bool(self.adam_w_mode))
                else:
                    for p in ps:
                        st = self.state[p]
                        reference.adam_update(p.data, st["exp_avg"], st["exp_avg_sq"], p.grad, group["lr"], beta1,
                                              beta2, group["eps"], group["weight_decay"], step,
                                              group["bias_correction"], bool(self.adam_w_mode))
        return loss
