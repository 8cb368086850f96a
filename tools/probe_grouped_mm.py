"""Probe: torch._grouped_mm on gfx950 (2D x 3D with offsets) — correctness vs per-expert matmul and timing vs the
in-tree grouped MFMA kernel at Mixtral shapes."""
import os, sys, time, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops import moe_ops

def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e3

E, H, N = 8, 4096, 28672
w = (torch.randn(E, N, H, device="cuda") / H**0.5).bfloat16()
for R in (32, 512, 4096, 16384):
    counts = torch.bincount(torch.randint(0, E, (R,), device="cuda"), minlength=E).int()
    offs = counts.cumsum(0).int()
    x = torch.randn(R, H, device="cuda").bfloat16()
    try:
        y = torch._grouped_mm(x, w.transpose(1, 2), offs=offs)
        ref = moe_ops.grouped_gemm(x, w, counts)
        err = (y.float() - ref.float()).abs().max().item()
        t_g = timeit(lambda: torch._grouped_mm(x, w.transpose(1, 2), offs=offs))
    except Exception as e:
        print("grouped_mm failed:", repr(e)[:300]); err, t_g = None, None
    t_k = timeit(lambda: moe_ops.grouped_gemm(x, w, counts))
    fl = 2 * R * N * H
    print(json.dumps({"R": R, "N": N, "K": H, "err": err, "torch_grouped_mm_ms": t_g, "kernel_ms": round(t_k, 3),
                      "torch_tflops": None if t_g is None else round(fl / t_g / 1e9, 1),
                      "kernel_tflops": round(fl / t_k / 1e9, 1)}), flush=True)
