"""RMSNorm forward / backward kernels at the Llama-2-7B step shape (32768 x 4096 bf16, residual fused): time per
call and effective HBM TB/s of the minimal traffic (fwd: read x, r; write y, x+r. bwd: read x, dy, dres; write dx).
One JSON line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


T, H = 32768, 4096
x, r, dy, dres = (torch.randn(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(4))
w = torch.ones(H, device="cuda", dtype=torch.bfloat16)
y, h, rstd = hip_ops().rms_fwd(x, r, w, 1e-5)
nb = T * H * 2
tf = timeit(lambda: hip_ops().rms_fwd(x, r, w, 1e-5))
tb = timeit(lambda: hip_ops().rms_bwd(dy, h, w, rstd, dres))
print(json.dumps({"rows": T, "H": H, "fwd_us": round(tf * 1e3, 1), "fwd_tbs": round(4 * nb / tf / 1e9, 2),
                  "bwd_us": round(tb * 1e3, 1), "bwd_tbs": round(4 * nb / tb / 1e9, 2)}), flush=True)
