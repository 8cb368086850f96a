#!/usr/bin/env python3
"""RMSNorm / LayerNorm backward (training path, residual fused) time and effective bandwidth per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    for H in (4096, 5120, 8192):
        for rows in (8192, 32768):
            x = torch.randn(rows, H, device="cuda").bfloat16().requires_grad_(True)
            r = torch.randn(rows, H, device="cuda").bfloat16().requires_grad_(True)
            w = torch.ones(H, device="cuda").bfloat16().requires_grad_(True)
            b = torch.zeros(H, device="cuda").bfloat16().requires_grad_(True)
            out = {}
            for name, fn in (("rms", lambda: DF.rms_norm(x, w, 1e-6, r)), ("ln", lambda: DF.layer_norm(x, w, b, 1e-5, r))):
                y, res = fn()
                gy, gr = torch.randn_like(y), torch.randn_like(res)
                for _ in range(3):
                    torch.autograd.grad((y, res), (x, r, w), (gy, gr), retain_graph=True)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    torch.autograd.grad((y, res), (x, r, w), (gy, gr), retain_graph=True)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 100
                # bytes: read dy, dres, x(normalised input); write dx (= dres_out): 4 x rows x H x 2 B
                out[name + "_bwd_us"] = round(us, 1)
                out[name + "_bwd_tb_s"] = round(4 * rows * H * 2 / (us * 1e-6) / 1e12, 2)
            print(json.dumps({"H": H, "rows": rows, **out}), flush=True)


if __name__ == "__main__":
    main()
