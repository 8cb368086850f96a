"""Flash backward ablation on MI355X (B8 H32 S4096 D128 causal): time the kernel with parts switched off through
DS_FLASH_BWD_DBG (1 no dQ atomics, 2 no dQ phase, 4 no dK/dV products, 8 no S/dP) to see where the time goes.
Results are timing-only (the outputs are wrong with any switch on). One JSON line per variant."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


B, Hq, Hk, S = 8, 32, 32, 4096
causal = len(sys.argv) < 2 or sys.argv[1] != "full"
q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
k = torch.randn(B, S, Hk, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
v = torch.randn(B, S, Hk, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
do = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
scale = 1 / math.sqrt(128)
o, lse = hip_ops().flash_fwd(q, k, v, causal, scale, True)
flops = 10 * B * Hq * S * S * 128 * (0.5 if causal else 1.0)
for dbg in (0, 1, 2, 4, 8, 2 | 4, 2 | 8, 4 | 8, 2 | 4 | 8):
    os.environ["DS_FLASH_BWD_DBG"] = str(dbg)
    t = timeit(lambda: hip_ops().flash_bwd(q, k, v, o, lse, do, scale, 1 if causal else 0))
    print(json.dumps({"dbg": dbg, "causal": causal, "ms": round(t, 3), "tflops_equiv": round(flops / t / 1e9, 1)}),
          flush=True)
