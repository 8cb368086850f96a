"""Hybrid engine (reference `tests/hybrid_engine/hybrid_engine_test.py`, `tests/unit/hybrid_engine/*`): train with
ZeRO and generate with the injected inference model on the same (updated) weights; LoRA fuse/unfuse round trip."""
import copy

import pytest
import torch

from ..common import run_distributed

transformers = pytest.importorskip("transformers")


def _hf_llama():
    torch.manual_seed(0)
    c = transformers.LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                 num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
    return transformers.LlamaForCausalLM(c)


class LoRALinear(torch.nn.Module):
    """DeepSpeed-Chat style LoRA linear with fuse/unfuse."""

    def __init__(self, base, r=4, scale=0.5):
        super().__init__()
        self.weight = base.weight
        self.bias = base.bias
        self.lora_right_weight = torch.nn.Parameter(torch.randn(base.in_features, r) * 0.1)
        self.lora_left_weight = torch.nn.Parameter(torch.randn(r, base.out_features) * 0.1)
        self.lora_scaling = scale
        self.fused = False

    def fuse_lora_weight(self):
        self.weight.data += self.lora_scaling * (self.lora_right_weight @ self.lora_left_weight).t()
        self.fused = True

    def unfuse_lora_weight(self):
        self.weight.data -= self.lora_scaling * (self.lora_right_weight @ self.lora_left_weight).t()
        self.fused = False

    def forward(self, x):
        y = torch.nn.functional.linear(x, self.weight, self.bias)
        if not self.fused:
            y = y + self.lora_scaling * (x @ self.lora_right_weight @ self.lora_left_weight)
        return y


def _run(stage, lora, tp, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.zero.partition_parameters import GatheredParameters
    model = _hf_llama()
    if lora:
        for layer in model.model.layers:
            layer.self_attn.q_proj = LoRALinear(layer.self_attn.q_proj)
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": stage},
           "hybrid_engine": {"enabled": True, "max_out_tokens": 64, "inference_tp_size": tp}}
    if lora:
        cfg["zero_optimization"]["stage"] = 0
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    ids = torch.randint(0, 128, (2, 8), generator=torch.Generator().manual_seed(3))
    results = []
    for it in range(2):
        got = eng.generate(ids, max_new_tokens=5)
        if it == 0 and stage < 3 and tp == 1:  # shared weights: the inference model aliases the training tensors
            ds_layer = eng._ds_model.layers[0]
            hf = eng.module.model.layers[0]
            assert ds_layer.o_w.data_ptr() == hf.self_attn.o_proj.weight.data_ptr()
            assert ds_layer.split_w["qkv_w"][0].data_ptr() == hf.self_attn.q_proj.weight.data_ptr()
            assert ds_layer.qkv_w.numel() == 0
        if tp > 1:
            assert eng._ds_model.tp_size == tp and eng._ds_model.layers[0].hq == 4 // tp
        # oracle: plain HF generate on a copy holding the gathered training weights (LoRA folded in)
        with GatheredParameters(list(eng.module.parameters())):
            ref_model = copy.deepcopy(eng.module)
        if lora:
            for m in ref_model.modules():
                if isinstance(m, LoRALinear):
                    m.fuse_lora_weight()
        ref = ref_model.generate(ids, max_new_tokens=5, do_sample=False)
        results.append((got, ref))
        x = torch.randint(0, 128, (2, 16), generator=torch.Generator().manual_seed(10 + it + dist.get_rank()))
        loss = eng(input_ids=x, labels=x).loss
        eng.backward(loss)
        eng.step()
    if lora:  # unfuse restored the training weights exactly
        for m in eng.module.modules():
            if isinstance(m, LoRALinear):
                assert not m.fused
    if dist.get_rank() == 0:
        torch.save(results, out)


@pytest.mark.parametrize("stage,lora,tp", [(3, False, 1), (2, False, 1), (0, True, 1), (3, False, 2), (2, False, 2)])
def test_hybrid_generate_tracks_training(stage, lora, tp, tmp_path):
    out = str(tmp_path / "h.pt")
    run_distributed(_run, 2, stage, lora, tp, out)
    results = torch.load(out, weights_only=True)
    for got, ref in results:
        assert torch.equal(got, ref)


def _per_layer(out):
    import deepspeedsyclsupport_amd as ds
    from ..inference.test_inference import tiny
    model = tiny("gpt2")
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 1},
           "hybrid_engine": {"enabled": True, "max_out_tokens": 64, "release_inference_cache": True}}
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    assert eng.create_inference_module() == model.config.num_hidden_layers
    assert type(eng._orig_modules[0]) in eng.inference_policies
    ids = torch.randint(0, model.config.vocab_size, (2, 10), generator=torch.Generator().manual_seed(5))
    diffs, moved = [], []
    prev = None
    for step in range(2):
        loss = eng(input_ids=ids, labels=ids).loss
        eng.backward(loss)
        eng.step()
        eng.eval()
        with torch.no_grad():
            ref = eng.module(ids, use_cache=False).logits.float()
            with eng.fused_layers() as conts:
                assert all(c.module.layer.qkv_w.numel() for c in conts)
                got = eng.module(ids, use_cache=False).logits.float()
            # forwards are the client's again, and the inference copies were released
            again = eng.module(ids, use_cache=False).logits.float()
        eng.train()
        assert all(c._released and c.module.layer.qkv_w.numel() == 0 for c in eng._inference_containers)
        diffs.append(float((got - ref).abs().max()))
        torch.testing.assert_close(again, ref)
        if prev is not None:
            moved.append(float((ref - prev).abs().max()))
        prev = ref
    eng.retake_inference_cache()
    assert all(not c._released and c.module.layer.qkv_w.numel() for c in eng._inference_containers)
    assert eng.convert_to_linear_transposed(model) is model
    torch.save({"diffs": diffs, "moved": moved}, out)


def test_per_layer_containers_track_training(tmp_path):
    """Layer containers built from `replace_policies`: inside `fused_layers()` the client layers run fused on the
    freshly trained weights; outside, the client forwards are back and the inference copies are released."""
    out = str(tmp_path / "r.pt")
    run_distributed(_per_layer, 1, out)
    r = torch.load(out, weights_only=True)
    assert max(r["diffs"]) < 2e-3 and r["moved"][0] > 10 * max(r["diffs"]), r
