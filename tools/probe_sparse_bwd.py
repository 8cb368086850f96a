"""Probe: efficient-attention backward with an additive layout bias (batch-expanded), fed with the block-sparse
forward's (O, LSE); errors vs an fp32 dense reference.

Finding (MI355X, torch 2.10 ROCm): the backward is exact when O has the [B, L, H, D] memory layout that both
SDPA and our flash kernels write; an O that is [B, H, L, D]-contiguous gives wrong dK/dV (dQ stays right) and,
with a batch-materialised bias, an illegal memory access. Only the safe layouts are exercised below."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.sparse_attention import block_sparse as bs
from deepspeedsyclsupport_amd.ops.sparse_attention.sparsity_config import FixedSparsityConfig
from deepspeedsyclsupport_amd.ops.native import hip_ops

torch.manual_seed(0)
B, H, L, D = 2, 4, 1024, 64
cfg = FixedSparsityConfig(num_heads=H, block=16, num_local_blocks=4)
layout = cfg.make_layout(L)
q, k, v = (torch.randn(B, H, L, D, device="cuda").bfloat16() for _ in range(3))
scale = D**-0.5
bias32 = bs.token_bias(layout, 16, L, H, torch.float32, "cuda")
qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
ref = torch.softmax((qr @ kr.transpose(-1, -2)) * scale + bias32, -1) @ vr
do = torch.randn_like(ref)
ref.backward(do)
tiles, ntiles, lay, qorder = bs.build_lut(layout, 16, L, q.device)
pad = lambda t: torch.nn.functional.pad(t, (0, 128 - D))
o, lse = hip_ops().flash_fwd_sparse(pad(q), pad(k), pad(v), scale, tiles, ntiles, qorder, lay, 16, True)
o = o[..., :D].contiguous()
print("fwd err", (o.float() - ref).abs().max().item())
z = torch.zeros((), dtype=torch.int64, device="cuda")
bias = bs.token_bias(layout, 16, L, H, torch.bfloat16, "cuda").expand(B, H, L, L)
so, sl, _, _ = torch.ops.aten._scaled_dot_product_efficient_attention(q, k, v, bias, True, 0.0, False, scale=scale)
print("o diff", (so.float() - o.float()).abs().max().item(), "o strides ours", o.stride(), "sdpa", so.stride())
print("lse diff", (sl[..., :L] - lse).abs().max().item(), "lse strides", lse.stride(), sl.stride(), tuple(sl.shape))
for name, oo, ll in (("o_sdpa+lse_ours", so, lse),
                     ("o_ours_tokmajor+lse_ours", o.transpose(1, 2).contiguous().transpose(1, 2), lse)):
    dq, dk, dv, _ = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
        do.bfloat16(), q, k, v, bias, oo, ll, z, z, 0.0, [True, True, True, False], False, scale=scale)
    torch.cuda.synchronize()
    print(name, "errs dq %.3f dk %.3f dv %.3f" % tuple(
        (a.float() - b.grad).abs().max().item() for a, b in ((dq, qr), (dk, kr), (dv, vr))), flush=True)
