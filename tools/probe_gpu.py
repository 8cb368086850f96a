"""Quick GPU capability probe: GEMM throughput via torch (hipBLASLt), SDPA backends, memory."""
import time, torch, torch.nn.functional as F
print("torch", torch.__version__, "hip", torch.version.hip, flush=True)
p = torch.cuda.get_device_properties(0)
print("dev", p.name, p.gcnArchName, "CUs", p.multi_processor_count, "mem GB", p.total_memory / 2**30, flush=True)

def bench(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters

for (m, n, k) in [(16384, 4096, 4096), (16384, 12288, 4096), (16384, 11008, 4096), (16384, 4096, 11008), (8192, 8192, 8192)]:
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16); b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    dt = bench(lambda: a @ b.t())
    print(f"gemm {m}x{n}x{k}: {2*m*n*k/dt/1e12:.0f} TF", flush=True)
for causal in (True, False):
    B, H, S, D = 4, 32, 4096, 128
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True); v = torch.randn_like(q, requires_grad=True)
    for name, be in [("flash", torch.nn.attention.SDPBackend.FLASH_ATTENTION), ("efficient", torch.nn.attention.SDPBackend.EFFICIENT_ATTENTION), ("math", torch.nn.attention.SDPBackend.MATH)]:
        try:
            with torch.nn.attention.sdpa_kernel([be]):
                dt = bench(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal), 5)
                fl = 4 * B * H * S * S * D * (0.5 if causal else 1)
                print(f"sdpa {name} causal={causal} fwd: {dt*1e3:.2f} ms {fl/dt/1e12:.0f} TF", flush=True)
                o = F.scaled_dot_product_attention(q, k, v, is_causal=causal); g = torch.randn_like(o)
                dt2 = bench(lambda: torch.autograd.grad(F.scaled_dot_product_attention(q, k, v, is_causal=causal), (q, k, v), g), 5)
                print(f"sdpa {name} causal={causal} fwd+bwd: {dt2*1e3:.2f} ms {3.5*fl/dt2/1e12:.0f} TF", flush=True)
        except Exception as e:
            print("sdpa", name, "failed", type(e).__name__, str(e)[:200], flush=True)
x = torch.empty(2**30, device="cuda", dtype=torch.uint8); y = torch.empty_like(x)
dt = bench(lambda: y.copy_(x)); print(f"copy bw {2*2**30/dt/1e12:.2f} TB/s", flush=True)
