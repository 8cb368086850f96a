"""DeepSpeedCPUAdam: host Adam for ZeRO-Offload / Offload++ (reference `deepspeed/ops/adam/cpu_adam.py`).

Backed by `ds_cpu_ops.cpu_adam_update` (target_clones AVX-512/AVX2 + OpenMP). `step(fp16_param_groups=...)` writes the
low-precision copy of each updated fp32 partition into the given (pinned) host tensors in the same pass, which the
ZeRO optimizer then ships to the GPU with an async H2D copy.
"""
import torch

from ..native import cpu_ops


class DeepSpeedCPUAdam(torch.optim.Optimizer):
    optimizer_id = 0

    def __init__(self, model_params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, adamw_mode=True, fp32_optimizer_states=True):
        if amsgrad:
            raise RuntimeError("DeepSpeedCPUAdam does not support AMSGrad")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, bias_correction=bias_correction,
                        amsgrad=amsgrad)
        super().__init__(model_params, defaults)
        self.opt_id = DeepSpeedCPUAdam.optimizer_id
        DeepSpeedCPUAdam.optimizer_id += 1
        self.adam_w_mode = adamw_mode
        self.fp32_optimizer_states = fp32_optimizer_states
        self.ds_opt_adam = cpu_ops()

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("amsgrad", False)

    @torch.no_grad()
    def step(self, closure=None, fp16_param_groups=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            for pi, p in enumerate(group["params"]):
                if p.grad is None:
                    continue
                assert p.device.type == "cpu", "CPUAdam param is on " + str(p.device)
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = 0
                    sd = torch.float32 if self.fp32_optimizer_states else p.dtype
                    state["exp_avg"] = torch.zeros_like(p.data, dtype=sd)
                    state["exp_avg_sq"] = torch.zeros_like(p.data, dtype=sd)
                state["step"] += 1
                b1, b2 = group["betas"]
                lp = None
                if fp16_param_groups is not None:
                    lp = fp16_param_groups[gi][pi] if isinstance(fp16_param_groups[gi], (list, tuple)) \
                        else fp16_param_groups[gi]
                    lp = lp.view(-1) if lp.device.type == "cpu" else None
                self.ds_opt_adam.cpu_adam_update(p.data.view(-1), state["exp_avg"].view(-1),
                                                 state["exp_avg_sq"].view(-1), p.grad.contiguous().view(-1), lp,
                                                 state["step"], group["lr"], b1, b2, group["eps"],
                                                 group["weight_decay"], group["bias_correction"], self.adam_w_mode,
                                                 1.0)
        return loss


def cpu_adam_flat_update(p, m, v, g, step, lr, beta1, beta2, eps, weight_decay, bias_correction=True,
                         adamw_mode=True, grad_scale=1.0, lp=None):
    cpu_ops().cpu_adam_update(p, m, v, g, lp, step, lr, beta1, beta2, eps, weight_decay, bias_correction, adamw_mode,
                              grad_scale)
