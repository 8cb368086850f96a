#!/usr/bin/env python3
"""Forward LayerNorm / RMSNorm latency at decode-sized row counts (one JSON line per case)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from deepspeedsyclsupport_amd.ops.transformer import functional as DF
    for H in (4096, 8192, 14336):
        for rows in [int(r) for r in os.environ.get("ROWS", "1,8,64,256,512,4096").split(",")]:
            x = torch.randn(rows, H, device="cuda").bfloat16()
            r = torch.randn(rows, H, device="cuda").bfloat16()
            g = torch.ones(H, device="cuda").bfloat16()
            b = torch.zeros(H, device="cuda").bfloat16()
            out = {}
            for name, fn in (("ln_res", lambda: DF.layer_norm(x, g, b, 1e-5, r)),
                             ("rms_res", lambda: DF.rms_norm(x, g, 1e-6, r))):
                with torch.no_grad():
                    for _ in range(5):
                        fn()
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        for _ in range(20):
                            fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        graph.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    out[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / 200, 2)
            print(json.dumps({"H": H, "rows": rows, **out}), flush=True)


if __name__ == "__main__":
    main()
