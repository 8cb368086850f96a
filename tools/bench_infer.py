#!/usr/bin/env python3
"""Llama-2-7B kernel-injected inference benchmark on one MI355X (random-init weights, synthetic prompts).

Reports prefill latency and decode throughput (tokens/s, ms/token) per batch size, eager vs HIP-graph decode.
    python tools/bench_infer.py --batches 1,16,64 --prompt 512 --gen 128
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
    ap.add_argument("--batches", default="1,16,64")
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--graph", default="0,1")
    ap.add_argument("--quant-bits", type=int, default=0, help="weight-only quantisation of the layer GEMMs (8 or 4); 16 = bf16 weights in the shuffled decode layout "
                    "(--group-size -1: keep a row-major copy for prefill too)")
    ap.add_argument("--group-size", type=int, default=128)
    args = ap.parse_args()
    from deepspeedsyclsupport_amd.inference.config import DeepSpeedInferenceConfig
    from deepspeedsyclsupport_amd.inference.engine import InferenceEngine
    from deepspeedsyclsupport_amd.inference.model_implementations.transformer import DSInferenceModel, DSModelSpec
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
    bf16_bytes = sum(p.numel() * 2 for layer in model.layers for p in layer.parameters() if p.dim() >= 2)
    stream_bytes = bf16_bytes
    if args.quant_bits == 32:  # row-major parameters + shuffled copies ("both")
        model.add_decode_layout()
    elif args.quant_bits:
        model.quantize_weights(args.quant_bits, args.group_size)
        torch.cuda.empty_cache()
        stream_bytes = sum(q.i8.nbytes() for layer in model.layers for q in layer.quant.values())
        if args.quant_bits in (16, 32):
            stream_bytes = bf16_bytes  # (a kept row-major copy is memory, not decode traffic)
    head_bytes = model.lm_head.numel() * 2
    for use_graph in [int(x) for x in args.graph.split(",")]:
        cfg = DeepSpeedInferenceConfig(dtype="bf16", enable_cuda_graph=bool(use_graph), max_tokens=4096)
        eng = InferenceEngine.__new__(InferenceEngine)
        torch.nn.Module.__init__(eng)
        eng._config, eng.dtype, eng.device, eng.injected, eng.module = cfg, torch.bfloat16, dev, True, model
        eng._graphs, eng.cuda_graph_created, eng.model_profile_enabled, eng._model_times = {}, False, False, []
        eng.tp_size, eng.tp_rank, eng.mp_group = 1, 0, None
        for B in [int(b) for b in args.batches.split(",")]:
            ids = torch.randint(0, 32000, (B, args.prompt), device=dev)
            eng.generate(ids, max_new_tokens=4)  # warm-up (+ graph capture)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.generate(ids, max_new_tokens=1)
            torch.cuda.synchronize()
            t_prefill = time.perf_counter() - t0
            t0 = time.perf_counter()
            eng.generate(ids, max_new_tokens=args.gen)
            torch.cuda.synchronize()
            t_all = time.perf_counter() - t0
            dec = max(t_all - t_prefill, 1e-9) / (args.gen - 1)
            print(json.dumps({"model": "Llama-2-7B", "batch": B, "prompt": args.prompt, "gen": args.gen,
                              "hip_graph": bool(use_graph), "prefill_ms": round(t_prefill * 1e3, 2),
                              "prefill_tok_s": round(B * args.prompt / t_prefill, 1),
                              "decode_ms_per_token": round(dec * 1e3, 3),
                              "decode_tok_s": round(B / dec, 1),
                              "weight_bits": 16 if args.quant_bits in (0, 16, 32) else args.quant_bits,
                              "group_size": args.group_size,
                              "decode_layout": {0: "row-major", 16: "shuffled", 32: "both"}.get(args.quant_bits, "packed"),
                              "layer_weight_gib_streamed": round(stream_bytes / 2**30, 3),
                              "lm_head_gib_bf16": round(head_bytes / 2**30, 3),
                              # bytes the decode step really reads (packed weights + scales + bf16 LM head) per second
                              "weight_stream_tb_s": round((stream_bytes + head_bytes) / dec / 1e12, 2),
                              # the same step priced at the bf16 model's bytes: what a bf16 decode would need to match
                              "bf16_equivalent_tb_s": round((bf16_bytes + head_bytes) / dec / 1e12, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
