"""Bias-path probe for flash_small: constant bias must be a no-op; a one-hot bias must select that key's V row."""
import torch

from deepspeedsyclsupport_amd.ops import flash_small as FS
from deepspeedsyclsupport_amd.ops.native import hip_ops

Z, S, H, D = 1, 128, 1, 32
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(Z, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
o0, _ = hip_ops().flash_small_fwd(q, k, v, None, None, 1, D**-0.5, 0.0, 0)
b1 = torch.full((Z, S), 3.0, device="cuda", dtype=torch.bfloat16)
o1, _ = hip_ops().flash_small_fwd(q, k, v, b1, None, 1, D**-0.5, 0.0, 0)
print("const bias diff", (o1.float() - o0.float()).abs().max().item(), flush=True)
for j in (0, 1, 2, 3, 4, 5, 8, 13, 31, 32, 33, 63, 64, 100):
    b1 = torch.full((Z, S), -30000.0, device="cuda", dtype=torch.bfloat16)
    b1[0, j] = 0
    o, _ = hip_ops().flash_small_fwd(q, k, v, b1, None, 1, D**-0.5, 0.0, 0)
    # which key's V does each query row return?
    d = (o[0, :, 0, None, :].float() - v[0, None, :, 0, :].float()).abs().amax(-1)  # [S, S]
    sel = d.argmin(-1)
    print(j, "selected keys (first 8 rows):", sel[:8].tolist(), "min err", d.min(-1).values.max().item(), flush=True)
for vec in (1, 0):
    for j in (0, 5):
        b2 = torch.full((Z, H, S, S), -30000.0, device="cuda", dtype=torch.bfloat16)
        b2[..., j] = 0
        o, _ = hip_ops().flash_small_fwd(q, k, v, None, b2, 1, D**-0.5, 0.0, 0)
        d = (o[0, :, 0, None, :].float() - v[0, None, :, 0, :].float()).abs().amax(-1)
        print("b2", j, d.argmin(-1)[:8].tolist(), flush=True)
    S2 = 126
    break
