"""Numerics probe for csrc/attn/flash_small.hip: prints the relative error of the forward for a ladder of cases."""
import torch

from deepspeedsyclsupport_amd.ops import flash_small as FS
from deepspeedsyclsupport_amd.ops.native import hip_ops


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


def run(Z, S, H, D, mode, b1=False, b2=False):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(Z, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    if mode == "zeroqk":
        q.zero_(); k.zero_()
    if mode == "eye":  # v = one-hot key index in column (key % D)
        v.zero_()
        for s in range(S):
            v[:, s, :, s % D] = 1.0
    bias1 = torch.randn(Z, S, device="cuda", generator=g).bfloat16() if b1 else None
    bias2 = torch.randn(Z, H, S, S, device="cuda", generator=g).bfloat16() if b2 else None
    o, lse = hip_ops().flash_small_fwd(q, k, v, bias1, bias2, 1, D**-0.5, 0.0, 0)
    torch.cuda.synchronize()
    ref = FS.reference(q, k, v, bias1, bias2)
    err = rel(o, ref)
    print(f"Z{Z} S{S} H{H} D{D} {mode:7s} b1={b1:d} b2={b2:d} rel={err:.4f}", flush=True)
    if err > 0.05:
        print("  o  ", o[0, :4, 0, :6].float().cpu().numpy().round(3).tolist())
        print("  ref", ref[0, :4, 0, :6].float().cpu().numpy().round(3).tolist())
        d = (o.float() - ref.float()).abs()
        print("  err by d  ", d.amax(dim=(0, 1, 2))[:D].cpu().numpy().round(2).tolist())
        print("  err by s  ", d.amax(dim=(0, 2, 3))[:64].cpu().numpy().round(2).tolist())


for D in (32, 64):
    for mode in ("zeroqk", "eye", "rand"):
        run(1, 64, 1, D, mode)
    run(2, 128, 3, D, "rand")
    run(2, 128, 3, D, "rand", b1=True)
    run(2, 128, 3, D, "rand", b2=True)
