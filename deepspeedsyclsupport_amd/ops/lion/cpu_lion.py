"""DeepSpeedCPULion (reference `deepspeed/ops/lion/cpu_lion.py`)."""
import torch

from ..native import cpu_ops


class DeepSpeedCPULion(torch.optim.Optimizer):
    optimizer_id = 0

    def __init__(self, model_params, lr=1e-3, betas=(0.9, 0.999), weight_decay=0, fp32_optimizer_states=True):
        super().__init__(model_params, dict(lr=lr, betas=betas, weight_decay=weight_decay))
        self.opt_id = DeepSpeedCPULion.optimizer_id
        DeepSpeedCPULion.optimizer_id += 1
        self.ds_opt_lion = cpu_ops()

    @torch.no_grad()
    def step(self, closure=None, fp16_param_groups=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            for pi, p in enumerate(group["params"]):
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p.data, dtype=torch.float32)
                st["step"] += 1
                lp = fp16_param_groups[gi][pi].view(-1) if fp16_param_groups is not None else None
                self.ds_opt_lion.cpu_lion_update(p.data.view(-1), st["exp_avg"].view(-1),
                                                 p.grad.contiguous().view(-1), lp, group["lr"], b1, b2,
                                                 group["weight_decay"], 1.0)
        return loss
