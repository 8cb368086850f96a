#!/usr/bin/env python3
"""Peak trainable parameters on ONE MI355X, and the Twin-Flow ratio sweep (the second half of the BASELINE metric:
"peak trainable params/GPU"; reference rows: >40 B on 1xV100-32GB + 1.5 TB host with ZeRO-3 Offload,
`docs/_posts/2021-03-08-zero3-offload.md:49`; Offload++ Twin-Flow speedup over ZeRO-Offload,
`blogs/deepspeed-offloadpp/README.md:10,34`).

Trains a Llama-architecture model (random init, synthetic tokens) with ZeRO-3 + ZeRO-Offload++ Twin-Flow over three
memory tiers. Per parameter (split masters: fp32 master = bf16 weight + int16 residual):
    device tier : 2 (weight) + 2 (residual) + 8 (moments) + 2 (grad)           = 14 B   (16 B with fp32 masters)
    host tier   : 2 on the device (weight) + 2 (residual) + 8 (moments) + 2 (pinned staging slot) on the host
    NVMe tier   : 2 on the device + 2 staging on the host + 10 B on disk (12 B with fp32 masters)
`--plan` solves the tier sizes from the three budgets. Every timed step is a full step: forward, backward (gradients
staged to the host on the d2h stream as they become final), device + host Adam concurrently, updated weights copied
back on the h2d stream. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

G = 2**30


def plan_tiers(n, split, device_gib, host_gib, disk_gib, act_gib=10.0):
    """Largest device tier that fits, then host, then NVMe: returns (ratio offloaded, elements resident on host,
    per-tier element counts, bytes) or raises if the model does not fit the three budgets."""
    mb = 2 if split else 4
    dev_state = mb + 8 + 2
    d = int(max(0.0, (device_gib - act_gib) * G - 2 * n) / dev_state)
    d = min(d, n)
    s = min(n - d, int(disk_gib * G / (mb + 8)))
    h = n - d - s
    host_need = h * (mb + 8 + 2) + s * 2
    if host_need > host_gib * G:
        # shrink nothing silently: the caller asked for a model that does not fit
        raise SystemExit(f"does not fit: device tier {d / 1e9:.2f}B, NVMe tier {s / 1e9:.2f}B, host tier "
                         f"{h / 1e9:.2f}B needs {host_need / G:.1f} GiB of host memory > {host_gib} GiB")
    return dict(ratio=(h + s) / n, max_in_cpu=h, device=d, host=h, nvme=s,
                device_gib=(2 * n + d * dev_state) / G, host_gib=host_need / G, disk_gib=s * (mb + 8) / G)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--inter", type=int, default=28672)
    ap.add_argument("--heads", type=int, default=64)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--layers", type=int, default=48)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--mb", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--ratio", type=float, default=None, help="offloaded fraction (default: planned from budgets)")
    ap.add_argument("--max-in-cpu", type=int, default=None, help="offloaded elements kept in DRAM (rest on NVMe)")
    ap.add_argument("--nvme-path", default=None)
    ap.add_argument("--no-split", action="store_true", help="separate fp32 master weights")
    ap.add_argument("--overlap-forward", action="store_true")
    ap.add_argument("--device-budget-gib", type=float, default=252.0)
    ap.add_argument("--host-budget-gib", type=float, default=250.0)
    ap.add_argument("--disk-budget-gib", type=float, default=0.0)
    ap.add_argument("--fresh-batches", action="store_true", help="new random tokens every step (default: one batch)")
    ap.add_argument("--tag", default="")
    ap.add_argument("--dry", action="store_true", help="print the plan only")
    args = ap.parse_args()

    from deepspeedsyclsupport_amd.models.llama import LlamaConfig
    cfg = LlamaConfig(vocab_size=32000, hidden_size=args.hidden, intermediate_size=args.inter,
                      num_hidden_layers=args.layers, num_attention_heads=args.heads,
                      num_key_value_heads=args.kv_heads, max_position_embeddings=args.seq)
    n = cfg.num_params()
    split = not args.no_split
    if args.ratio is None:
        plan = plan_tiers(n, split, args.device_budget_gib, args.host_budget_gib, args.disk_budget_gib)
        ratio, max_in_cpu = plan["ratio"], plan["max_in_cpu"]
    else:
        ratio = args.ratio
        max_in_cpu = args.max_in_cpu if args.max_in_cpu is not None else int(n * ratio)
        plan = dict(ratio=ratio, max_in_cpu=max_in_cpu)
    use_nvme = args.nvme_path is not None and max_in_cpu < int(n * ratio) - 1
    print(json.dumps({"params": n, "split_master": split, "plan": plan, "nvme": use_nvme}), file=sys.stderr,
          flush=True)
    if args.dry:
        return

    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.models.llama import LlamaForCausalLM
    ds.init_distributed(dist_backend="nccl")
    torch.cuda.set_device(0)
    t0 = time.time()
    stop = threading.Event()
    import psutil
    proc = psutil.Process()
    peak_rss = [0.0]

    def heartbeat():
        while not stop.wait(20):
            rss = proc.memory_info().rss / G
            peak_rss[0] = max(peak_rss[0], rss)
            print(f"[maxparams] alive {time.time() - t0:.0f}s gpu {torch.cuda.memory_allocated() / G:.1f} GiB "
                  f"host rss {rss:.1f} GiB", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg)
    torch.set_default_dtype(prev)
    model.gradient_checkpointing_enable()
    print(f"[maxparams] built {n / 1e9:.2f}B params in {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    zero = {"stage": 3, "sub_group_size": 64 * 2**20}
    if ratio > 0:
        oc = {"device": "nvme" if use_nvme else "cpu", "ratio": ratio, "pin_memory": True,
              "overlap_forward": args.overlap_forward}
        if use_nvme:
            oc.update(nvme_path=args.nvme_path, max_in_cpu=max_in_cpu)
        zero["offload_optimizer"] = oc
    conf = {
        "train_micro_batch_size_per_gpu": args.mb, "steps_per_print": 10**9,
        "bf16": {"enabled": True, "split_master_weights": split}, "gradient_clipping": 1.0,
        "optimizer": {"type": "AdamW", "params": {"lr": args.lr, "betas": [0.9, 0.95], "weight_decay": 0.1}},
        "zero_optimization": zero,
        "aio": {"block_size": 8 * 2**20, "queue_depth": 8, "thread_count": 2},
    }
    engine, _, _, _ = ds.initialize(model=model, config=conf)
    opt = engine.optimizer
    off = opt.off
    tiers = {"device": int(sum(m.numel() for m in opt.master)),
             "host": int(sum(off.res)) if off else 0,
             "nvme": int(sum(off.n) - sum(off.res)) if off else 0}
    print(f"[maxparams] engine ready {time.time() - t0:.0f}s gpu {torch.cuda.memory_allocated() / G:.1f} GiB "
          f"tiers {json.dumps(tiers)}", file=sys.stderr, flush=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randint(0, cfg.vocab_size, (args.mb, args.seq), device="cuda", generator=g)
    times, losses = [], []
    for i in range(args.steps + 1):
        if args.fresh_batches:
            x = torch.randint(0, cfg.vocab_size, (args.mb, args.seq), device="cuda", generator=g)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        loss = engine(x, labels=x)
        engine.backward(loss)
        engine.step()
        if i == args.steps:
            opt.join_offload()  # the last step's host update is part of the measurement
        torch.cuda.synchronize()
        dt = time.perf_counter() - ts
        losses.append(float(loss.detach()))
        if i > 0:
            times.append(dt)
        print(f"[maxparams] step {i} {dt:.1f}s loss {losses[-1]:.4f} norm {opt.get_global_grad_norm():.3f}",
              file=sys.stderr, flush=True)
    stop.set()
    peak_rss[0] = max(peak_rss[0], proc.memory_info().rss / G)
    step_s = sum(times) / len(times)
    toks = args.mb * args.seq / step_s
    out = {"metric": "peak trainable params / MI355X (ZeRO-3 + Offload++ Twin-Flow)", "params": n,
           "params_billion": round(n / 1e9, 2), "offloaded_ratio": round(ratio, 4), "tiers_params": tiers,
           "split_master_weights": split, "overlap_forward": args.overlap_forward, "n_gpus": 1,
           "seq_len": args.seq, "micro_batch": args.mb, "step_s": round(step_s, 2),
           "step_times_s": [round(t, 2) for t in times], "tokens_per_s": round(toks, 1),
           "model_tflops": round(toks * cfg.flops_per_token(args.seq) / 1e12, 1),
           "peak_gpu_mem_gib": round(torch.cuda.max_memory_allocated() / G, 1),
           "peak_host_rss_gib": round(peak_rss[0], 1),
           "nvme_gib": round(opt.nvme_swapper.bytes_on_disk() / G, 1) if opt.nvme_swapper else 0.0,
           "losses": [round(v, 4) for v in losses], "dtype": "bf16",
           "data": "synthetic tokens (" + ("fresh batch per step" if args.fresh_batches else
                                          "one batch repeated") + "), random init",
           "config": {"hidden": args.hidden, "inter": args.inter, "heads": args.heads, "kv_heads": args.kv_heads,
                      "layers": args.layers, "activation_checkpointing": True, "lr": args.lr}, "tag": args.tag}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
