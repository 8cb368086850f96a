"""1-bit Adam (reference `runtime/fp16/onebit/adam.py:14-306`).

Warm-up (step < freeze_step): plain Adam on data-parallel averaged gradients. After that the second moment is
frozen and ranks stop all-reducing gradients: each updates its momentum with its LOCAL gradient and the momentum is
averaged with the error-compensated 1-bit all-reduce (`runtime/comm/compressed.py`) — 1/32 of the bytes. Under the
flat-group ZeRO engine the optimizer sees one flat fp32 tensor per parameter group, so each step is ONE compressed
collective per group. As in the reference, no bias correction is applied to the update.
"""
import torch

from ...comm.compressed import CompressedBackend


class OnebitAdam(torch.optim.Optimizer):

    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, bias_correction=True,
                 betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0,
                 amsgrad=False, cuda_aware=False, comm_backend_name="nccl"):
        if amsgrad:
            raise RuntimeError("1-bit Adam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.deepspeed = deepspeed
        self.freeze_step = freeze_step
        self.adam_freeze_key = False
        self.initialize = False
        self.comm_backend_name = comm_backend_name
        self.comm_in_optimizer = True
        self._backend = None
        self._step = 0

    def backend(self):
        if self._backend is None:
            group = getattr(self.deepspeed, "seq_data_parallel_group", None) if self.deepspeed is not None else None
            self._backend = CompressedBackend(group)
        return self._backend

    def skip_grad_allreduce(self):
        """True once the variance is frozen: gradients stay local and momentum is compressed-averaged instead."""
        return self.adam_freeze_key

    @torch.no_grad()
    def step(self, closure=None, grads=None):
        loss = closure() if closure is not None else None
        compress = self.adam_freeze_key
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
                st["step"] += 1
                m, v = st["exp_avg"], st["exp_avg_sq"]
                if not compress:
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                    m.mul_(b1).add_(g, alpha=1 - b1)
                else:
                    if "worker_error" not in st:
                        be = self.backend()
                        n = be.padded_size(p.numel())
                        st["worker_error"] = torch.zeros(n, dtype=torch.float32, device=p.device)
                        st["server_error"] = torch.zeros(n // be.world, dtype=torch.float32, device=p.device)
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    self.backend().compressed_allreduce(m, st["worker_error"], st["server_error"])
                if self.eps_mode == 0:
                    upd = m / (v + group["eps"]).sqrt()
                else:
                    upd = m / (v.sqrt() + group["eps"])
                if group["weight_decay"] > 0:
                    upd = upd + group["weight_decay"] * p.float()
                p.add_(upd.to(p.dtype), alpha=-group["lr"])
        self._step += 1
        if not self.adam_freeze_key and self._step >= self.freeze_step:
            self.adam_freeze_key = True  # the next backward keeps gradients local
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._step = max((s.get("step", 0) for s in self.state.values()), default=0)
        self.adam_freeze_key = self._step >= self.freeze_step
        for s in self.state.values():  # error feedback restarts after a reload (reference behaviour)
            s.pop("worker_error", None)
            s.pop("server_error", None)
