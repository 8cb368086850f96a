#!/usr/bin/env python3
"""Inference v2 ragged step on one MI355X: Llama-2-7B architecture (random-init bf16 weights, synthetic tokens).

A FastGen-style step mixes D running decodes (context C) with one SplitFuse prompt chunk of P tokens:
  * ragged : ONE `put()` over the D + P concatenated tokens (one forward, paged decode + paged flash prefill);
  * split  : the previous engine's schedule — one forward for the decodes, one for the chunk.
Also a pure-decode step and a pure-chunk step for reference. Prints one JSON line per (D, P).
    python tools/bench_ragged.py --decodes 32 --context 512 --chunks 256,512 --iters 10
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decodes", type=int, default=32)
    ap.add_argument("--context", type=int, default=512)
    ap.add_argument("--chunks", default="128,512")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--layers", type=int, default=32)
    args = ap.parse_args()
    from deepspeedsyclsupport_amd.inference.model_implementations.transformer import DSInferenceModel, DSModelSpec
    from deepspeedsyclsupport_amd.inference.v2 import AllocationMode, InferenceEngineV2, RaggedInferenceEngineConfig
    dev = torch.device("cuda", 0)
    spec = DSModelSpec(arch="llama", vocab_size=32000, hidden_size=4096, num_layers=args.layers, num_heads=32,
                       num_kv_heads=32, intermediate_size=11008, norm="rms", norm_eps=1e-5, pos="rope",
                       max_positions=4096)
    torch.manual_seed(0)
    model = DSInferenceModel(spec, dtype=torch.bfloat16, device=dev)
    with torch.no_grad():
        for p in model.parameters():
            if p.dim() >= 2:
                p.normal_(0, 0.02)
    cfg = RaggedInferenceEngineConfig(state_manager={"memory_config": {"mode": AllocationMode.ALLOCATE, "size": 4096},
                                                     "max_ragged_batch_size": 8192, "max_ragged_sequence_count": 512,
                                                     "max_tracked_sequences": 512, "max_context": 8192},
                                      kv_cache={"block_size": 64})
    eng = InferenceEngineV2(model, cfg)
    D, C = args.decodes, args.context
    g = torch.Generator().manual_seed(0)
    # D running sequences with C cached tokens each
    for u in range(D):
        eng.put([u], [torch.randint(0, 32000, (C, ), generator=g)])
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.iters

    uid = [10_000]
    dec_tok = [torch.randint(0, 32000, (1, ), generator=g) for _ in range(D)]

    def new_prompt_uid():
        uid[0] += 1
        return uid[0]

    for P in [int(c) for c in args.chunks.split(",")]:
        chunk = torch.randint(0, 32000, (P, ), generator=g)

        def ragged():
            u = new_prompt_uid()
            eng.put(list(range(D)) + [u], dec_tok + [chunk])
            eng.flush(u)

        def split():
            u = new_prompt_uid()
            eng.put(list(range(D)), dec_tok)
            eng.put([u], [chunk])
            eng.flush(u)

        def decode_only():
            eng.put(list(range(D)), dec_tok)

        def chunk_only():
            u = new_prompt_uid()
            eng.put([u], [chunk])
            eng.flush(u)

        t_r, t_s, t_d, t_c = timed(ragged), timed(split), timed(decode_only), timed(chunk_only)
        print(json.dumps({"model": "Llama-2-7B", "decodes": D, "context": C, "chunk": P,
                          "ragged_step_ms": round(t_r * 1e3, 2), "split_step_ms": round(t_s * 1e3, 2),
                          "decode_only_ms": round(t_d * 1e3, 2), "chunk_only_ms": round(t_c * 1e3, 2),
                          "ragged_tok_s": round((D + P) / t_r, 1), "split_tok_s": round((D + P) / t_s, 1),
                          "data": "synthetic tokens, random-init weights"}), flush=True)
        # the decode sequences grew by (iters + 1) * 3 tokens per P; keep contexts bounded
    for u in range(D):
        eng.flush(u)


if __name__ == "__main__":
    main()
