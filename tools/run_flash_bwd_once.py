"""Runs the gfx950 flash backward a few times at one shape (for rocprofv3 counter passes)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402

B, Hq, Hk, S = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (8, 32, 32, 4096)))
causal = True
q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
k = torch.randn(B, S, Hk, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
v = torch.randn(B, S, Hk, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
do = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
o, lse = hip_ops().flash_fwd(q, k, v, causal, 128**-0.5, True)
for _ in range(3):
    hip_ops().flash_bwd(q, k, v, o, lse, do, 128**-0.5, 1)
torch.cuda.synchronize()
print("done")
