"""Hypothesis probe for the flash backward's dQ: which product does the kernel's dq match? (S=64, one head)"""
import sys

import torch

sys.path.insert(0, ".")
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402

torch.manual_seed(0)
S = 64
q, k, v, do = (torch.randn(1, 1, S, 128, device="cuda", dtype=torch.bfloat16) for _ in range(4))
scale = 128**-0.5
o, lse = hip_ops().flash_fwd(q, k, v, False, scale, True)
dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, scale, 0)
Q, K, V, dO = (t[0, 0].float() for t in (q, k, v, do))
P = torch.softmax(Q @ K.T * scale, -1)
dP = dO @ V.T
dS = P * (dP - (P * dP).sum(-1, keepdim=True))
ours = dq[0, 0].float()


def corr(name, cand):
    c = torch.corrcoef(torch.stack([ours.flatten(), cand.flatten()]))[0, 1].item()
    r = (ours.norm() / cand.norm()).item()
    print(f"{name:40s} corr={c:+.4f} norm_ratio={r:.4f}", flush=True)


corr("ref dS@K*scale", dS @ K * scale)
corr("P@K*scale", P @ K * scale)
corr("dS@K", dS @ K)
corr("slab0 only", dS[:, :32] @ K[:32] * scale)
corr("slab1 only", dS[:, 32:] @ K[32:] * scale)
corr("dS^T@K (key/q swapped)", dS.T @ K * scale)
for name, perm in (("keys 4-blocks reversed", torch.arange(64).view(-1, 4).flip(-1).flatten()),
                   ("keys swap 4<->8 halves", torch.arange(64).view(-1, 2, 2, 4).transpose(1, 2).flatten()),
                   ("keys swap 8-blocks in 16", torch.arange(64).view(-1, 2, 8).flip(1).flatten())):
    corr(name, dS[:, perm] @ K * scale)
    corr(name + " (K perm)", dS @ K[perm] * scale)
for name, perm in (("q rows 4-blocks swap (4h)", torch.arange(64).view(-1, 2, 2, 4).transpose(1, 2).flatten()),):
    corr(name, (dS @ K * scale)[perm])
print("ours[0,:4]", ours[0, :4].tolist(), "ref", (dS @ K * scale)[0, :4].tolist())
print("ours rows norm", ours.norm(dim=1)[:8].tolist())
print("ref rows norm", (dS @ K * scale).norm(dim=1)[:8].tolist())
