#!/usr/bin/env python3
"""Run the int8 skinny GEMM MFMA path (pre-shuffled weights) a few times at one shape (for rocprofv3 passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepspeedsyclsupport_amd.ops.native import hip_ops  # noqa: E402

N, K, M = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (57344, 14336, 8)))
qsh = torch.randint(-127, 127, ((N + 15) // 16, K // 64, 64, 16), dtype=torch.int8, device="cuda")
ssh = torch.rand((N + 15) // 16, K // 64, 16, device="cuda") * 0.01
x = torch.randn(M, K, device="cuda").bfloat16()
for _ in range(10):
    hip_ops().skinny_i8_sh(x, qsh, ssh, None, N, 64)
torch.cuda.synchronize()
print("ok")
