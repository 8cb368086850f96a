"""Flash-attention backward micro-benchmark on MI355X: the in-tree gfx950 backward (csrc/attn/flash_bwd.hip) vs the
library efficient-attention backward that round 1 used (aiter via aten::_scaled_dot_product_efficient_attention_backward),
Llama-2-7B / 70B shapes. Prints one JSON line per config; FLOPs counted as 10*B*Hq*S^2*D (x0.5 causal)."""
import json
import math
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


CONFIGS = [(8, 32, 32, 4096, True), (8, 32, 32, 4096, False), (4, 64, 8, 4096, True), (1, 32, 32, 16384, True),
           (1, 4, 4, 32768, True)]
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    CONFIGS = CONFIGS[:1]

for (B, Hq, Hk, S, causal) in CONFIGS:
    q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    k = torch.randn(B, S, Hk, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    v = torch.randn(B, S, Hk, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    do = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    scale = 1 / math.sqrt(128)
    o, lse = hip_ops().flash_fwd(q, k, v, causal, scale, True)
    flops = 10 * B * Hq * S * S * 128 * (0.5 if causal else 1.0)
    t_ours = timeit(lambda: hip_ops().flash_bwd(q, k, v, o, lse, do, scale, 1 if causal else 0))
    res = {"B": B, "Hq": Hq, "Hk": Hk, "S": S, "causal": causal, "ours_ms": round(t_ours, 3),
           "ours_tflops": round(flops / t_ours / 1e9, 1)}
    try:
        rep = Hq // Hk
        z = torch.zeros((), dtype=torch.int64, device="cuda")

        def lib():
            ke = k.repeat_interleave(rep, 1) if rep > 1 else k
            ve = v.repeat_interleave(rep, 1) if rep > 1 else v
            return torch.ops.aten._scaled_dot_product_efficient_attention_backward(
                do, q, ke, ve, None, o, lse, z, z, 0.0, [True, True, True, False], causal, scale=scale)
        t = timeit(lib)
        res["library_ms"] = round(t, 3)
        res["library_tflops"] = round(flops / t / 1e9, 1)
    except Exception as e:  # noqa: BLE001
        res["library"] = f"unavailable: {e}"[:100]
    print(json.dumps(res), flush=True)
    del q, k, v, do, o, lse
    torch.cuda.empty_cache()

if len(sys.argv) > 1 and sys.argv[1] == "quick":
    # pre / post passes alone (delta + zeroing, dq conversion): same traffic as inside flash_bwd
    B, Hq, S = 8, 32, 4096
    o = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    acc = torch.empty(B * Hq * S * 128, device="cuda", dtype=torch.float32)
    t = timeit(lambda: (o.float() * o.float()).sum(-1))
    t0 = timeit(lambda: acc.zero_())
    print(json.dumps({"zero_dqacc_ms": round(t0, 3), "torch_delta_ms": round(t, 3)}), flush=True)
