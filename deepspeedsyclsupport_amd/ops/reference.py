"""Plain-PyTorch fp32 reference implementations.

Used (1) as the numerics oracle in tests of the HIP kernels and (2) for host (CPU) tensors on the gloo plumbing
path. Device tensors never come here (see `ops/native.py`).
"""
import math

import torch
import torch.nn.functional as F


def adam_update(p, m, v, g, lr, beta1, beta2, eps, wd, step, bias_correction=True, adamw=True, grad_scale=1.0,
                lp=None):
    gf = g.float() * grad_scale
    pf = p.float()
    if not adamw and wd != 0:
        gf = gf + wd * pf
    mf = m.float().mul_(beta1).add_(gf, alpha=1 - beta1)
    vf = v.float().mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    bc1 = 1 - beta1**step if bias_correction else 1.0
    bc2 = 1 - beta2**step if bias_correction else 1.0
    denom = vf.sqrt() / math.sqrt(bc2) + eps
    upd = (mf / bc1) / denom
    if adamw and wd != 0:
        upd = upd + wd * pf
    pf = pf - lr * upd
    p.copy_(pf)
    m.copy_(mf)
    v.copy_(vf)
    if lp is not None:
        lp.copy_(pf)


def lion_update(p, m, g, lr, beta1, beta2, wd, grad_scale=1.0, lp=None):
    gf = g.float() * grad_scale
    pf = p.float()
    mf = m.float()
    c = beta1 * mf + (1 - beta1) * gf
    pf = pf * (1 - lr * wd) - lr * torch.sign(c)
    mf = beta2 * mf + (1 - beta2) * gf
    p.copy_(pf)
    m.copy_(mf)
    if lp is not None:
        lp.copy_(pf)


def adagrad_update(p, s, g, lr, eps, wd, grad_scale=1.0, lp=None):
    gf = g.float() * grad_scale
    pf = p.float()
    if wd != 0:
        gf = gf + wd * pf
    sf = s.float() + gf * gf
    pf = pf - lr * gf / (sf.sqrt() + eps)
    p.copy_(pf)
    s.copy_(sf)
    if lp is not None:
        lp.copy_(pf)


def lamb_update(p, m, v, g, lr, beta1, beta2, eps, wd, step, bias_correction=True, grad_scale=1.0, max_coeff=10.0,
                min_coeff=0.01, lp=None):
    gf = g.float() * grad_scale
    pf = p.float()
    mf = m.float().mul_(beta1).add_(gf, alpha=1 - beta1)
    vf = v.float().mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    bc1 = 1 - beta1**step if bias_correction else 1.0
    bc2 = 1 - beta2**step if bias_correction else 1.0
    u = (mf / bc1) / ((vf / bc2).sqrt() + eps) + wd * pf
    wn, un = pf.norm(), u.norm()
    trust = (wn / un) if (wn > 0 and un > 0) else torch.tensor(1.0)
    trust = float(min(max(float(trust), min_coeff), max_coeff))
    pf = pf - lr * trust * u
    p.copy_(pf)
    m.copy_(mf)
    v.copy_(vf)
    if lp is not None:
        lp.copy_(pf)
    return trust


def rms_norm(x, w, eps, residual=None):
    h = x.float() + residual.float() if residual is not None else x.float()
    y = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype), (h.to(x.dtype) if residual is not None else None)


def layer_norm(x, g, b, eps, residual=None):
    h = x.float() + residual.float() if residual is not None else x.float()
    y = F.layer_norm(h, (h.shape[-1], ), g.float(), b.float(), eps)
    return y.to(x.dtype), (h.to(x.dtype) if residual is not None else None)


ACTS = {0: F.silu, 1: lambda x: F.gelu(x, approximate="tanh"), 2: F.gelu, 3: F.relu, 4: lambda x: x}


def gated_act(gu, act=0):
    g, u = gu.float().chunk(2, dim=-1)
    return (ACTS[act](g) * u).to(gu.dtype)


def rope_tables(max_pos, rot, base=10000.0, scaling=None, device=None):
    inv = 1.0 / (base**(torch.arange(0, rot, 2, dtype=torch.float64) / rot))
    t = torch.arange(max_pos, dtype=torch.float64)
    if scaling:
        t = t / scaling
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def apply_rope_half(x, cos, sin, pos):
    """x [B, S, H, D] (rotate_half on the first 2*cos.shape[-1] dims); pos [S] or [B,S] long."""
    rot = cos.shape[-1] * 2
    c = cos[pos].float()
    s = sin[pos].float()
    if c.dim() == 2:
        c, s = c[None, :, None, :], s[None, :, None, :]
    else:
        c, s = c[:, :, None, :], s[:, :, None, :]
    xf = x.float()
    x1, x2, rest = xf[..., :rot // 2], xf[..., rot // 2:rot], xf[..., rot:]
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    return torch.cat([o1, o2, rest], dim=-1).to(x.dtype)


def cross_entropy(logits, labels, ignore_index=-100, smoothing=0.0):
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index, reduction="none",
                           label_smoothing=smoothing)
