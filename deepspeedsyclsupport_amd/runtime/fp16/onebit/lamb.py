"""1-bit LAMB (reference `runtime/fp16/onebit/lamb.py:14-443`; Li et al., "1-bit LAMB").

Warm-up: LAMB on averaged gradients, recording each tensor's trust ratio (lamb coefficient) as an EMA
(coeff_beta). After freeze_step the variance and the base coefficient are frozen; momentum is updated from local
gradients and averaged with the 1-bit all-reduce, and the frozen coefficient is rescaled each step by the ratio of
the fresh update's norm to the frozen-variance update's norm, clamped to [factor_min, factor_max] and to a
factor_threshold change per step, then bounded by [min_coeff, max_coeff].
"""
import torch

from ...comm.compressed import CompressedBackend


class OnebitLamb(torch.optim.Optimizer):

    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, bias_correction=True,
                 betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0,
                 max_coeff=10.0, min_coeff=0.01, amsgrad=False, cuda_aware=False, comm_backend_name="nccl",
                 coeff_beta=0.9, factor_max=4.0, factor_min=0.5, factor_threshold=0.1):
        if amsgrad:
            raise RuntimeError("1-bit LAMB does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm, max_coeff=max_coeff, min_coeff=min_coeff)
        super().__init__(params, defaults)
        self.deepspeed = deepspeed
        self.freeze_step = freeze_step
        self.coeff_beta = coeff_beta
        self.factor_max, self.factor_min, self.factor_threshold = factor_max, factor_min, factor_threshold
        self.lamb_freeze_key = False
        self.comm_in_optimizer = True
        self._backend = None
        self._step = 0

    def backend(self):
        if self._backend is None:
            group = getattr(self.deepspeed, "seq_data_parallel_group", None) if self.deepspeed is not None else None
            self._backend = CompressedBackend(group)
        return self._backend

    def skip_grad_allreduce(self):
        return self.lamb_freeze_key

    @torch.no_grad()
    def step(self, closure=None, grads=None):
        loss = closure() if closure is not None else None
        frozen = self.lamb_freeze_key
        for group in self.param_groups:
            b1, b2 = group["betas"]
            eps, wd = group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad.float()
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    st["lamb_coeff_freeze"] = 0.0
                    st["last_factor"] = 1.0
                st["step"] += 1
                m, v = st["exp_avg"], st["exp_avg_sq"]
                w = p.float()
                wnorm = w.norm()
                if not frozen:
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                    upd = m / (v.sqrt() + eps)
                    if wd > 0:
                        upd = upd + wd * w
                    unorm = upd.norm()
                    coeff = (wnorm / unorm).clamp(group["min_coeff"], group["max_coeff"]).item() \
                        if wnorm > 0 and unorm > 0 else 1.0
                    st["lamb_coeff_freeze"] = (self.coeff_beta * st["lamb_coeff_freeze"] +
                                               (1 - self.coeff_beta) * coeff)
                else:
                    if "worker_error" not in st:
                        be = self.backend()
                        n = be.padded_size(p.numel())
                        st["worker_error"] = torch.zeros(n, dtype=torch.float32, device=p.device)
                        st["server_error"] = torch.zeros(n // be.world, dtype=torch.float32, device=p.device)
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    self.backend().compressed_allreduce(m, st["worker_error"], st["server_error"])
                    upd = m / (v.sqrt() + eps)
                    if wd > 0:
                        upd = upd + wd * w
                    # fresh second moment estimate from the synchronised momentum -> scaling factor
                    v_fresh = b2 * v + (1 - b2) * m * m
                    upd_fresh = m / (v_fresh.sqrt() + eps)
                    factor = (upd.norm() / upd_fresh.norm().clamp_min(1e-12)).item()
                    factor = min(max(factor, self.factor_min), self.factor_max)
                    lo, hi = st["last_factor"] * (1 - self.factor_threshold), \
                        st["last_factor"] * (1 + self.factor_threshold)
                    factor = min(max(factor, lo), hi)
                    st["last_factor"] = factor
                    coeff = min(max(st["lamb_coeff_freeze"] * factor, group["min_coeff"]), group["max_coeff"])
                p.add_((upd * coeff).to(p.dtype), alpha=-group["lr"])
        self._step += 1
        if not self.lamb_freeze_key and self._step >= self.freeze_step:
            self.lamb_freeze_key = True
        return loss

    def get_lamb_coeffs(self):
        return [self.state[p].get("lamb_coeff_freeze", 0.0) for g in self.param_groups for p in g["params"]]
