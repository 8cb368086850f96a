"""0/1 Adam (reference `runtime/fp16/onebit/zoadam.py:14-359`; Lu et al., "Maximizing Communication Efficiency for
Large-scale Training via 0/1 Adam").

All communication is 1-bit: gradients are never all-reduced in full precision.
  * variance: refreshed only at exponentially spaced steps (interval x var_update_scaler after every refresh) until
    var_freeze_step, from the 1-bit-averaged gradient;
  * momentum: updated from the local gradient; parameters take local steps, and the accumulated update is
    synchronised with the 1-bit all-reduce every `local_step` steps, the interval doubling (local_step_scaler) up to
    local_step_clipper once the variance is frozen.
"""
import torch

from ...comm.compressed import CompressedBackend


class ZeroOneAdam(torch.optim.Optimizer):

    def __init__(self, params, deepspeed=None, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0, var_freeze_step=100000,
                 var_update_scaler=16, local_step_scaler=32678, local_step_clipper=16, amsgrad=False,
                 cuda_aware=False, comm_backend_name="nccl"):
        if amsgrad:
            raise RuntimeError("0/1 Adam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.deepspeed = deepspeed
        self.var_freeze_step = var_freeze_step
        self.var_update_scaler = var_update_scaler
        self.local_step_scaler = local_step_scaler
        self.local_step_clipper = local_step_clipper
        self.comm_in_optimizer = True
        self.freeze_key = False
        self._backend = None
        self._step = 0
        self._var_interval = 1
        self._next_var_update = 0
        self._local_interval = 1
        self._next_sync = 0

    def backend(self):
        if self._backend is None:
            group = getattr(self.deepspeed, "seq_data_parallel_group", None) if self.deepspeed is not None else None
            self._backend = CompressedBackend(group)
        return self._backend

    def skip_grad_allreduce(self):
        return True

    def _errors(self, st, p, key):
        if key not in st:
            be = self.backend()
            n = be.padded_size(p.numel())
            st[key] = (torch.zeros(n, dtype=torch.float32, device=p.device),
                       torch.zeros(n // be.world, dtype=torch.float32, device=p.device))
        return st[key]

    @torch.no_grad()
    def step(self, closure=None, grads=None):
        loss = closure() if closure is not None else None
        t = self._step
        var_update = (not self.freeze_key) and t >= self._next_var_update
        sync = t >= self._next_sync
        be = self.backend()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad.float()
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    st["anchor"] = p.detach().float().clone()  # params at the last synchronisation
                st["step"] += 1
                m, v = st["exp_avg"], st["exp_avg_sq"]
                if var_update:
                    ga = g.clone()
                    we, se = self._errors(st, p, "grad_err")
                    be.compressed_allreduce(ga, we, se)
                    v.mul_(b2).addcmul_(ga, ga, value=1 - b2)
                m.mul_(b1).add_(g, alpha=1 - b1)
                denom = (v + group["eps"]).sqrt() if self.eps_mode == 0 else v.sqrt().add_(group["eps"])
                upd = m / denom
                if group["weight_decay"] > 0:
                    upd = upd + group["weight_decay"] * p.float()
                p.add_(upd.to(p.dtype), alpha=-group["lr"])
                if sync:
                    # average the drift accumulated since the last sync (1-bit), then re-anchor
                    delta = p.float() - st["anchor"]
                    we, se = self._errors(st, p, "delta_err")
                    be.compressed_allreduce(delta, we, se)
                    p.copy_((st["anchor"] + delta).to(p.dtype))
                    st["anchor"].copy_(p.float())
                    mw, ms = self._errors(st, p, "mom_err")
                    be.compressed_allreduce(m, mw, ms)
        if var_update:
            self._next_var_update = t + self._var_interval
            self._var_interval *= self.var_update_scaler
        if sync:
            if self.freeze_key:
                self._local_interval = min(self._local_interval * 2, self.local_step_clipper)
            self._next_sync = t + self._local_interval
        self._step += 1
        if not self.freeze_key and self._step >= self.var_freeze_step:
            self.freeze_key = True
        return loss
