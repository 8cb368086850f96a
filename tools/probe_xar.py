#!/usr/bin/env python3
"""Two ranks on one GPU: print what the xGMI all-reduce returns for tiny messages (debug aid)."""
import os
import sys

import torch
import torch.distributed as tdist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank = int(os.environ["RANK"])
    tdist.init_process_group("gloo")
    torch.cuda.set_device(0)
    from deepspeedsyclsupport_amd.comm.xgmi import XgmiAllReduce
    ar = XgmiAllReduce(None, cap_bytes=4 << 20)
    for dt in (torch.float32, torch.bfloat16):
        for n in (8, 16, 64):
            for mode in (1, 2):
                t = (torch.arange(n, dtype=torch.float32) + 100 * (rank + 1)).to(dt).cuda()
                y = ar.all_reduce(t.clone(), mode=mode)
                torch.cuda.synchronize()
                ref = (torch.arange(n, dtype=torch.float32) * 2 + 300)
                bad = (y.float().cpu() - ref).abs().max().item()
                print(f"rank {rank} {dt} n={n} mode={mode} maxerr={bad} y[:16]={y.float().cpu()[:16].tolist()}",
                      flush=True)
    print(f"rank {rank} err word {ar.error()}", flush=True)
    tdist.barrier()
    ar.close()


if __name__ == "__main__":
    main()
