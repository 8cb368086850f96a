"""Diagnostic for the gfx950 flash backward: per-tensor max error of dq / dk / dv against fp32 autograd on a few
small shapes (prints one JSON line per case)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402


def ref(q, k, v, causal, scale):
    rep = q.shape[1] // k.shape[1]
    kk = k.repeat_interleave(rep, 1)
    vv = v.repeat_interleave(rep, 1)
    s = (q @ kk.transpose(-1, -2)) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ vv


for (B, Hq, Hk, S, causal) in [(1, 1, 1, 256, False), (1, 1, 1, 256, True), (1, 1, 1, 64, False),
                               (1, 2, 1, 512, True), (2, 4, 4, 512, True)]:
    torch.manual_seed(0)
    q = torch.randn(B, Hq, S, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, 128, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B, Hq, S, 128, device="cuda", dtype=torch.bfloat16)
    scale = 128**-0.5
    o, lse = hip_ops().flash_fwd(q, k, v, causal, scale, True)
    dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, scale, 1 if causal else 0)
    q32, k32, v32 = (t.float().requires_grad_() for t in (q, k, v))
    ref(q32, k32, v32, causal, scale).backward(do.float())
    res = {"B": B, "Hq": Hq, "Hk": Hk, "S": S, "causal": causal}
    for n, a, b in (("dq", dq, q32.grad), ("dk", dk, k32.grad), ("dv", dv, v32.grad)):
        e = (a.float() - b).abs()
        res[n] = [round(e.max().item(), 4), round(b.abs().max().item(), 4)]
        # where the error sits: per 32-row tile of the sequence and per 32-column slab of D
        res[n + "_rows"] = [round(x, 3) for x in e[0, 0].reshape(-1, 32, 128).amax((1, 2)).tolist()[:8]]
        res[n + "_cols"] = [round(x, 3) for x in e[0, 0].reshape(S, 4, 32).amax((0, 2)).tolist()]
    # ratio test: is dq a scaled / transposed version of the reference?
    res["dq_ratio_med"] = round((dq.float() / q32.grad).median().item(), 4)
    print(json.dumps(res), flush=True)
