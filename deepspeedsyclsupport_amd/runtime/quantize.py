"""MoQ: quantize-aware training in the optimizer step (reference `runtime/quantize.py:14` `Quantizer`, driven from
`runtime/engine.py:1384-1401` `_configure_quantization` and `:2069-2079` after `optimizer.step()`).

After every optimizer step the 16-bit working weights of the compress layers are replaced by their fake-quantised
values (the fp32 masters keep full precision, so the quantisation noise never accumulates in the optimizer). Each
weight carries its own schedule — `start_bits`, `target_bits`, `q_period` (set by
`compression.basic_layer.LinearLayer_Compress.enable_weight_quantization`) — and drops one bit every time the step
count passes its period, doubling the period (times the eigenvalue factor when the Hessian-eigenvalue schedule is on)
each time. With `fp16_mixed_quantize` the weights are blended `ratio * w + (1 - ratio) * q(w)` with the ratio
falling by `quantize_change_ratio` per step, so the switch to the quantised weights is gradual.

Bit widths >= 3 use group-wise symmetric/asymmetric rounding (nearest or stochastic); 2 bits is the ternary
quantiser (threshold 0.7 * mean |w|, per-group scale alpha), 1 bit the binary one (sign * mean |w|). With
`quantizer_kernel` the >= 3-bit path runs the gfx950 quantize/dequantize kernels (`ops/quantizer`) in place.
"""
import math

import torch

from ..utils.logging import logger

TWO_D_PARAMS = 6  # the reference's count of 2-D weights per transformer block, used to look one step ahead


class Quantizer:

    def __init__(self, q_groups=1, q_mixed_fp16=False, q_change_ratio=0.01, q_type="symmetric", q_rounding="nearest",
                 q_verbose=False, q_eigenvalue=False, use_quantizer_kernel=False, layer_num=0):
        self.q_groups = max(int(q_groups), 1)
        self.q_mixed_fp16 = bool(q_mixed_fp16)
        self.q_change_ratio = float(q_change_ratio)
        self.q_type = q_type
        self.q_rounding = q_rounding
        self.q_verbose = q_verbose
        self.q_eigenvalue = q_eigenvalue
        self.use_quantizer_kernel = use_quantizer_kernel
        self.layer_num = layer_num
        self.qsteps = 0
        self.quantize_real_ratio = 1.0
        self._params = []  # weights seen by the last quantize() call (for any_precision_switch)

    # ------------------------------------------------------------------------------------------ schedule
    def any_precision_switch(self):
        """Will any weight drop a bit within the next block-sized window of steps? The engine recomputes the
        Hessian eigenvalues only then (they only matter when a period is stretched)."""
        if self.layer_num == 0:
            return True
        horizon = self.qsteps + TWO_D_PARAMS * self.layer_num
        return any(p.start_bits != p.target_bits and horizon >= p.q_period for p in self._params)

    def step(self):
        self.qsteps += 1

    def update_fp16_ratio(self):
        if self.q_mixed_fp16:
            self.quantize_real_ratio = max(self.quantize_real_ratio - self.q_change_ratio, 0.0)

    def _advance_bits(self, p, index, factor):
        if p.start_bits != p.target_bits and self.qsteps >= p.q_period:
            self.quantize_real_ratio = 1.0
            p.q_period = (p.q_period << 1) * factor
            p.start_bits -= 1
            if self.q_verbose:
                logger.info(f"MoQ: weight {index} now {p.start_bits} bits at step {self.qsteps}, "
                            f"next period {p.q_period}")
        if p.start_bits < p.target_bits:
            raise ValueError(f"MoQ: bit width {p.start_bits} fell below the target {p.target_bits}")

    # ------------------------------------------------------------------------------------------ quantisers
    def _groups(self, w):
        g = self.q_groups if w.numel() % self.q_groups == 0 else 1
        return w.reshape(g, -1)

    def quantize_highbit(self, w, bits):
        x = self._groups(w.float())
        levels = 2**bits
        noise = 0.0 if self.q_rounding == "nearest" else torch.empty_like(x).uniform_(-0.5, 0.5)
        if self.q_type == "symmetric":
            amax = x.abs().amax(dim=1, keepdim=True)
            scale = (2 * amax / levels).clamp_min(1e-12)
            y = torch.clamp(torch.round(x / scale + noise), -(levels >> 1), (levels >> 1) - 1) * scale
        else:
            lo, hi = x.amin(dim=1, keepdim=True), x.amax(dim=1, keepdim=True)
            scale = ((hi - lo) / levels).clamp_min(1e-12)
            zp = torch.round(lo / scale) * scale
            y = torch.clamp(torch.round((x - zp) / scale + noise), 0, levels - 1) * scale + zp
        return y.reshape(w.shape)

    def quantize_tenary(self, w):
        x = self._groups(w.float())
        thres = 0.7 * x.abs().mean(dim=1, keepdim=True)
        keep = (x.abs() > thres).float()
        alpha = (keep * x.abs()).sum(dim=1, keepdim=True) / keep.sum(dim=1, keepdim=True).clamp_min(1.0)
        return (alpha * torch.sign(x) * keep).reshape(w.shape)

    def quantize_binary(self, w):
        x = self._groups(w.float())
        return (torch.sign(x) * x.abs().mean(dim=1, keepdim=True)).reshape(w.shape)

    def compute_quantization(self, p, index=0, factor=1):
        self._advance_bits(p, index, factor)
        bits = p.start_bits
        w = p.data
        if bits <= 2 and (self.q_type != "symmetric" or self.q_rounding != "nearest"):
            raise ValueError("MoQ ternary/binary quantisation needs symmetric, nearest rounding")
        if self.use_quantizer_kernel and w.is_cuda and bits >= 3:
            from ..ops.quantizer import quantizer as Q
            gs = w.numel() // (self.q_groups if w.numel() % self.q_groups == 0 else 1)
            # the kernels pack 4- and 8-bit codes; other widths round on the next wider grid's math in torch
            if bits in (4, 8) and gs % 2 == 0:
                qt = Q.quantize(w, gs, bits, symmetric=self.q_type == "symmetric",
                                stochastic_rounding=self.q_rounding != "nearest", seed=self.qsteps)
                q = Q.dequantize(qt, torch.float32)
            else:
                q = self.quantize_highbit(w, bits)
        elif bits >= 3:
            q = self.quantize_highbit(w, bits)
        elif bits == 2:
            q = self.quantize_tenary(w)
        else:
            q = self.quantize_binary(w)
        if self.q_mixed_fp16 and bits >= p.target_bits - 1:
            q = self.quantize_real_ratio * w.float() + (1.0 - self.quantize_real_ratio) * q
        return q

    @torch.no_grad()
    def quantize(self, parameter_group, overflow, eigenvalue_enabled, block_eigenvalue=None):
        """Quantise every MoQ-scheduled weight of `parameter_group` (list of lists of params) in place. Skipped on an
        fp16 overflow step unless the eigenvalue schedule is on (reference semantics)."""
        if overflow and not eigenvalue_enabled:
            return
        self.step()
        self.update_fp16_ratio()
        self._params = []
        for group in parameter_group:
            for p in group:
                if p.dim() < 2 or not getattr(p, "start_bits", None):
                    continue
                self._params.append(p)
                ev, layer_id = (None, 0)
                if block_eigenvalue:
                    ev, layer_id = block_eigenvalue.get(id(p), (None, 0))
                factor = 1 + math.floor(ev * 4) if ev is not None else 1
                # in place: the working weights may be views into a flat ZeRO buffer
                p.data.copy_(self.compute_quantization(p, layer_id, factor).to(p.dtype))
