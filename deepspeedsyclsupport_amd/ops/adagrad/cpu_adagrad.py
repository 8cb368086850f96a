"""DeepSpeedCPUAdagrad (reference `deepspeed/ops/adagrad/cpu_adagrad.py`)."""
import torch

from ..native import cpu_ops


class DeepSpeedCPUAdagrad(torch.optim.Optimizer):
    optimizer_id = 0

    def __init__(self, model_params, lr=1e-2, eps=1e-10, weight_decay=0, amsgrad=False, fp32_optimizer_states=True):
        super().__init__(model_params, dict(lr=lr, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad))
        self.opt_id = DeepSpeedCPUAdagrad.optimizer_id
        DeepSpeedCPUAdagrad.optimizer_id += 1
        self.fp32_optimizer_states = fp32_optimizer_states
        self.ds_opt_adagrad = cpu_ops()

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
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg_sq"] = torch.zeros_like(p.data, dtype=torch.float32)
                st["step"] += 1
                if p.grad.is_sparse:
                    g = p.grad.to_dense()
                else:
                    g = p.grad
                lp = None
                if fp16_param_groups is not None:
                    lp = fp16_param_groups[gi][pi].view(-1)
                self.ds_opt_adagrad.cpu_adagrad_update(p.data.view(-1), st["exp_avg_sq"].view(-1),
                                                       g.contiguous().view(-1), lp, group["lr"], group["eps"],
                                                       group["weight_decay"], 1.0)
        return loss
