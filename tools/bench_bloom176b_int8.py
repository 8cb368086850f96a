#!/usr/bin/env python3
"""BLOOM-176B weight-only-int8 kernel-injected inference on ONE MI355X (BASELINE config "BLOOM-176B
transformer_inference kernel-inject TP=8, int8 quantizer"; the reference needs 8 GPUs, 288 GB of HBM holds the
whole int8 model on one).

The real BLOOM-176B architecture (70 layers, hidden 14336, 112 heads, vocab 250880, ALiBi, LayerNorm, GELU) with
random-init weights: built on the meta device and materialised ONE layer at a time on the GPU (random bf16 ->
group-int8 quantised -> bf16 freed), so the 352 GB bf16 model never exists. Decode steps run the fused-dequant
int8 skinny GEMV (`csrc/gemv/skinny_int8.hip`) and the paged-KV decode attention; prefill dequantises per GEMM.
Prints one JSON line per batch size.
    python tools/bench_bloom176b_int8.py --layers 70 --batches 1,8 --prompt 128 --gen 32
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build(layers, dev, bits=8, group=64):
    from deepspeedsyclsupport_amd.inference.model_implementations.transformer import (DSInferenceModel, DSModelSpec,
                                                                                    alibi_slopes)
    spec = DSModelSpec(arch="bloom", vocab_size=250880, hidden_size=14336, num_layers=layers, num_heads=112,
                       num_kv_heads=112, intermediate_size=4 * 14336, norm="ln", norm_eps=1e-5, pos="alibi",
                       act="gelu_tanh", gated_mlp=False, qkv_bias=True, o_bias=True, mlp_bias=True, embed_norm=True,
                       tie_embeddings=True, max_positions=2048)
    model = DSInferenceModel(spec, dtype=torch.bfloat16, device=torch.device("meta"))
    g = torch.Generator(device=dev).manual_seed(0)

    # top-level params (embedding tied to the LM head, as in BLOOM)
    model.to_empty(device=dev, recurse=False)
    with torch.no_grad():
        model.embed.normal_(0, 0.02, generator=g)
        model.lm_head.data = model.embed.data
        model.embed_ln_w.fill_(1.0)
        model.embed_ln_b.zero_()
        model.norm_w.fill_(1.0)
        model.norm_b.zero_()
        if model.lm_head_b is not None:
            model.lm_head_b.zero_()
    model.alibi = alibi_slopes(spec.num_heads).to(dev)
    t0 = time.time()
    for i, layer in enumerate(model.layers):
        layer.to_empty(device=dev)
        with torch.no_grad():
            for name, p in layer.named_parameters():
                if p.dim() >= 2:
                    p.normal_(0, 0.02, generator=g)
                elif name.endswith("_w") and name.startswith("ln"):
                    p.fill_(1.0)
                else:
                    p.zero_()
        layer.quantize_weights(bits, group)
        if i % 10 == 0:
            log(f"[bloom] layer {i}/{layers} quantised, {torch.cuda.memory_allocated() / 2**30:.1f} GiB, "
                f"{time.time() - t0:.1f}s")
    model.device = dev
    return model, spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=70)
    ap.add_argument("--batches", default="1,8")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--gen", type=int, default=32)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--bits", type=int, default=8, choices=(4, 8))
    ap.add_argument("--group", type=int, default=64)
    args = ap.parse_args()
    from deepspeedsyclsupport_amd.inference.config import DeepSpeedInferenceConfig
    from deepspeedsyclsupport_amd.inference.engine import InferenceEngine
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, spec = build(args.layers, dev, args.bits, args.group)
    n_q = sum(layer.quant[n].shape.numel() for layer in model.layers for n in layer.quant)
    weights_gib = torch.cuda.memory_allocated() / 2**30
    log(f"[bloom] built: {n_q / 1e9:.1f}B int{args.bits} layer params + embedding, {weights_gib:.1f} GiB on device")
    cfg = DeepSpeedInferenceConfig(dtype="bf16", enable_cuda_graph=bool(args.graph), max_tokens=args.prompt + args.gen)
    eng = InferenceEngine.from_ds_model(model, cfg)
    for B in [int(b) for b in args.batches.split(",")]:
        ids = torch.randint(0, spec.vocab_size, (B, args.prompt), device=dev)
        eng.generate(ids, max_new_tokens=3)  # warm-up (+ graph capture)
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
        print(json.dumps({"model": "BLOOM-176B" if args.layers == 70 else f"BLOOM-176B-{args.layers}L",
                          "weights": f"int{args.bits} weight-only (group {args.group}) + bf16 embedding", "n_gpus": 1, "tp": 1,
                          "batch": B, "prompt": args.prompt, "gen": args.gen, "hip_graph": bool(args.graph),
                          "device_weights_gib": round(weights_gib, 1),
                          "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                          "prefill_ms": round(t_prefill * 1e3, 1), "decode_ms_per_token": round(dec * 1e3, 2),
                          "decode_tok_s": round(B / dec, 1),
                          "weight_stream_tb_s": round(weights_gib * 2**30 / dec / 1e12, 2),
                          "data": "synthetic prompts, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
