"""Single-rank rehearsal of the multi-GPU ZeRO path: DS_ZERO_FORCE_PARTITION=1 turns on the partitioned code (flat
shards, all-gather on the ag stream, reduce-scatter on the rs stream, ZeRO-3 fetch/release/prefetch) with one rank.
The loss trajectory must match the LOCAL (dp == 1) path for ZeRO-1/2/3. Runs on CPU (gloo) or on one GPU (RCCL).

    MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 python tools/zero_rehearsal_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.unit.simple_model import base_config, tiny_llama  # noqa: E402
import deepspeedsyclsupport_amd as ds  # noqa: E402


def run(stage, force, steps=5):
    os.environ["DS_ZERO_FORCE_PARTITION"] = "1" if force else "0"
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    torch.manual_seed(0)
    m = tiny_llama(hidden_size=128, intermediate_size=256, num_attention_heads=4)
    cfg = base_config(stage=stage, lr=3e-3, mb=2, clip=1.0, dtype="fp32")
    cfg["zero_optimization"].update({"stage3_param_persistence_threshold": 0})
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(steps):
        x = torch.randint(0, 128, (2, 32), generator=g).to(dev)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        out.append(float(loss))
    return out


if __name__ == "__main__":
    worst = 0.0
    for st in (1, 2, 3):
        a, b = run(st, False), run(st, True)
        d = max(abs(x - y) for x, y in zip(a, b))
        worst = max(worst, d)
        print(f"stage {st}: local {[round(v, 5) for v in a]} forced {[round(v, 5) for v in b]} max|diff| {d:.2e}")
    sys.exit(0 if worst < 2e-3 else 1)
