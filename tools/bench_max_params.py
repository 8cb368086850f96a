#!/usr/bin/env python3
"""Peak trainable parameters on ONE MI355X (the second half of the BASELINE metric: "peak trainable params/GPU";
reference rows: >40 B on 1xV100-32GB + 1.5 TB host with ZeRO-3 Offload, 13 B with ZeRO-Offload,
`docs/_posts/2021-03-08-zero3-offload.md:49`).

Trains a Llama-architecture model (random init, synthetic tokens) with ZeRO-3 + ZeRO-Offload++ Twin-Flow: a
`ratio` fraction of the fp32 master weights and Adam moments lives in (exact-size pinned) host memory and is stepped by
the native CPU Adam concurrently with the fused HIP Adam on the device part. The ratio is solved from the two memory
budgets (HBM and the host RAM this job may use), per parameter:
    device: 2 (bf16 weight) + 2 (bf16 grad) + (1 - r) * 12 (fp32 master + 2 moments)
    host:   r * 18 (pinned fp32 master + fp32 grad + bf16 copy, 2 fp32 moments)
Every timed step is a full step (forward, backward, device + host Adam, H2D of the host-updated weights).
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=6144)
    ap.add_argument("--inter", type=int, default=16384)
    ap.add_argument("--heads", type=int, default=48)
    ap.add_argument("--layers", type=int, default=50)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--mb", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--ratio", type=float, default=None, help="Twin-Flow host fraction (default: solved)")
    ap.add_argument("--device-budget-gib", type=float, default=245.0)
    ap.add_argument("--host-budget-gib", type=float, default=170.0)
    ap.add_argument("--dry", action="store_true", help="print the plan only")
    args = ap.parse_args()

    from deepspeedsyclsupport_amd.models.llama import LlamaConfig
    cfg = LlamaConfig(vocab_size=32000, hidden_size=args.hidden, intermediate_size=args.inter,
                      num_hidden_layers=args.layers, num_attention_heads=args.heads, max_position_embeddings=args.seq)
    n = cfg.num_params()
    G = 2**30
    dev_b, host_b = args.device_budget_gib * G, args.host_budget_gib * G
    if args.ratio is None:
        r_min = max(0.0, (16 * n - dev_b) / (12 * n))  # smallest host share that fits the device
        r = min(1.0, r_min + 0.02)
    else:
        r = args.ratio
    dev_need, host_need = n * (4 + 12 * (1 - r)), n * 18 * r
    plan = {"params": n, "ratio": round(r, 4), "device_state_gib": round(dev_need / G, 1),
            "host_state_gib": round(host_need / G, 1)}
    print(json.dumps({"plan": plan}), file=sys.stderr, flush=True)
    if host_need > host_b or dev_need > dev_b:
        raise SystemExit(f"does not fit the budgets: {plan}")
    if args.dry:
        return

    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.models.llama import LlamaForCausalLM
    ds.init_distributed(dist_backend="nccl")
    torch.cuda.set_device(0)
    t0 = time.time()
    stop = threading.Event()

    def heartbeat():
        while not stop.wait(30):
            print(f"[maxparams] alive {time.time() - t0:.0f}s gpu {torch.cuda.memory_allocated() / G:.1f} GiB",
                  file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg)
    torch.set_default_dtype(prev)
    model.gradient_checkpointing_enable()
    print(f"[maxparams] built {n / 1e9:.2f}B params in {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    conf = {
        "train_micro_batch_size_per_gpu": args.mb, "steps_per_print": 10**9, "bf16": {"enabled": True},
        "gradient_clipping": 1.0,
        "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "betas": [0.9, 0.95], "weight_decay": 0.1}},
        "zero_optimization": {"stage": 3, "offload_optimizer": {"device": "cpu", "ratio": r, "pin_memory": True}},
    }
    engine, _, _, _ = ds.initialize(model=model, config=conf)
    print(f"[maxparams] engine ready {time.time() - t0:.0f}s gpu {torch.cuda.memory_allocated() / G:.1f} GiB",
          file=sys.stderr, flush=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    times, losses = [], []
    for i in range(args.steps + 1):
        x = torch.randint(0, cfg.vocab_size, (args.mb, args.seq), device="cuda", generator=g)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        loss = engine(x, labels=x)
        engine.backward(loss)
        engine.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - ts
        losses.append(float(loss.detach()))
        if i > 0:
            times.append(dt)
        print(f"[maxparams] step {i} {dt:.1f}s loss {losses[-1]:.3f}", file=sys.stderr, flush=True)
    stop.set()
    import psutil
    rss = psutil.Process().memory_info().rss / G
    step_s = sum(times) / len(times)
    toks = args.mb * args.seq / step_s
    out = {"metric": "peak trainable params / MI355X (ZeRO-3 + Offload++ Twin-Flow)", "params": n,
           "params_billion": round(n / 1e9, 2), "twin_flow_ratio": round(r, 4), "n_gpus": 1,
           "seq_len": args.seq, "micro_batch": args.mb, "step_s": round(step_s, 2), "tokens_per_s": round(toks, 1),
           "model_tflops": round(toks * cfg.flops_per_token(args.seq) / 1e12, 1),
           "peak_gpu_mem_gib": round(torch.cuda.max_memory_allocated() / G, 1), "host_rss_gib": round(rss, 1),
           "losses": [round(v, 4) for v in losses], "dtype": "bf16", "data": "synthetic tokens, random init",
           "config": {"hidden": args.hidden, "inter": args.inter, "heads": args.heads, "layers": args.layers,
                      "activation_checkpointing": True}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
