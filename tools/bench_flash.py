"""Flash-attention forward micro-benchmark on MI355X: in-tree gfx950 kernel vs SDPA (efficient / flash backends),
Llama-2-7B shape (B x 32 heads x S x 128, causal and not). Prints one JSON line per config."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from torch.nn.attention import SDPBackend, sdpa_kernel  # noqa: E402

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


for (B, H, S) in [(4, 32, 4096), (8, 32, 4096), (1, 32, 16384), (1, 4, 32768)]:
    for causal in (True, False):
        q, k, v = (torch.randn(B, H, S, 128, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        scale = 1 / math.sqrt(128)
        flops = 4 * B * H * S * S * 128 * (0.5 if causal else 1.0)
        t_ours = timeit(lambda: hip_ops().flash_fwd(q, k, v, causal, scale, True))
        res = {"B": B, "H": H, "S": S, "causal": causal, "ours_ms": round(t_ours, 3),
               "ours_tflops": round(flops / t_ours / 1e9, 1)}
        for name, be in (("sdpa_efficient", SDPBackend.EFFICIENT_ATTENTION), ("sdpa_flash", SDPBackend.FLASH_ATTENTION)):
            try:
                with sdpa_kernel([be]):
                    t = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal))
                res[name + "_ms"] = round(t, 3)
                res[name + "_tflops"] = round(flops / t / 1e9, 1)
            except Exception as e:  # noqa: BLE001
                res[name] = f"unavailable: {e}"[:80]
        print(json.dumps(res), flush=True)
        del q, k, v
