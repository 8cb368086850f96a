"""Megatron checkpoint re-sharding at load time and the ds_model descriptor path of init_inference (reference
`runtime/state_dict_factory.py`, `runtime/weight_quantizer.py`, `tests/unit/inference/test_checkpoint_sharding.py`).

No Megatron checkpoint ships with the reference, so the fixtures are synthetic: a full-size "global" state dict is
cut into P model-parallel files with Megatron's layouts, and a job at degree M must get exactly the slices a
degree-M writer would have produced."""
import json

import pytest
import torch

from deepspeedsyclsupport_amd.runtime.state_dict_factory import MegatronSDLoader, SDLoaderFactory
from deepspeedsyclsupport_amd.runtime.weight_quantizer import WeightQuantization

H, HEADS, HN, L = 16, 4, 4, 2


def _global_sd(seed=0):
    g = torch.Generator().manual_seed(seed)
    sd = {"word_embeddings.weight": torch.randn(32, H, generator=g),
          "position_embeddings.weight": torch.randn(8, H, generator=g),
          "transformer.final_layernorm.weight": torch.randn(H, generator=g)}
    for i in range(L):
        p = f"transformer.layers.{i}."
        # fused QKV as [3, heads, hn] blocks (for version 0) — the head-major versions use [heads, 3, hn]
        sd[p + "attention.query_key_value.weight"] = torch.randn(3 * HEADS * HN, H, generator=g)
        sd[p + "attention.query_key_value.bias"] = torch.randn(3 * HEADS * HN, generator=g)
        sd[p + "attention.dense.weight"] = torch.randn(H, HEADS * HN, generator=g)
        sd[p + "attention.dense.bias"] = torch.randn(H, generator=g)
        sd[p + "mlp.dense_h_to_4h.weight"] = torch.randn(4 * H, H, generator=g)
        sd[p + "mlp.dense_h_to_4h.bias"] = torch.randn(4 * H, generator=g)
        sd[p + "mlp.dense_4h_to_h.weight"] = torch.randn(H, 4 * H, generator=g)
        sd[p + "mlp.dense_4h_to_h.bias"] = torch.randn(H, generator=g)
        sd[p + "input_layernorm.weight"] = torch.randn(H, generator=g)
    return sd


def _shard(sd, P, r, ver):
    """What a Megatron writer at degree P stores on rank r."""
    out = {}
    for k, v in sd.items():
        if "query_key_value" in k:
            if ver == 0:  # [3, heads, hn]: rank r keeps heads r*heads/P.. of each of q, k, v
                out[k] = torch.cat([b.chunk(P, 0)[r] for b in v.chunk(3, 0)], 0)
            else:  # head-major: a contiguous block of heads
                out[k] = v.chunk(P, 0)[r]
        elif "attention.dense.weight" in k or "dense_4h_to_h.weight" in k:
            out[k] = v.chunk(P, 1)[r]
        elif "dense_h_to_4h" in k or "word_embeddings" in k:
            out[k] = v.chunk(P, 0)[r]
        else:
            out[k] = v
    return out


def _write(tmp_path, sd, P, ver):
    files = []
    for r in range(P):
        f = tmp_path / f"mp_rank_{r:02d}_model_states.pt"
        torch.save({"module": _shard(sd, P, r, ver), "checkpoint_version": ver, "mp_world_size": P}, f)
        files.append(str(f))
    return files


@pytest.mark.parametrize("ver", [0, 2.0])
@pytest.mark.parametrize("P,M", [(4, 2), (4, 1), (2, 4), (1, 2), (2, 2)])
def test_megatron_reshard_matches_direct_writer(tmp_path, P, M, ver):
    sd = _global_sd()
    files = _write(tmp_path, sd, P, ver)
    loader = SDLoaderFactory.get_sd_loader_json({"type": "Megatron", "checkpoints": files, "version": None})
    assert isinstance(loader, MegatronSDLoader)
    for r in range(M):
        _, got, (scales, count) = loader.load(M, r)
        assert scales is None and count == (P // M if P > M else 1)
        want = _shard(sd, M, r, ver)
        for k, v in want.items():
            torch.testing.assert_close(got["module"][k], v, rtol=0, atol=0, msg=k)


def test_weight_quantization_roundtrip_and_scale_table():
    wq = WeightQuantization(mlp_extra_grouping=True, mp_size=1)
    sd = {k: v for k, v in _global_sd().items() if "layers.0." in k}
    ref = {k: v.clone() for k, v in sd.items()}
    qsd, table = wq.sd_quantize_megatron(sd, 8, 4)
    assert table.shape[0] == 1 and table.shape[1] == 4  # one layer x (qkv, dense, h4h, 4hh)
    key = "transformer.layers.0.mlp.dense_h_to_4h.weight"
    assert qsd[key].dtype == torch.int8
    # MLP weights get twice the groups; dequantised values within one step of the originals (the reference grid
    # 2^b / (2 amax) puts +amax one step past the largest code)
    s = table[0, 2, :8].reshape(8, 1)
    deq = (qsd[key].float().reshape(8, -1) * s).reshape(ref[key].shape)
    assert (deq - ref[key]).abs().max() <= s.max() + 1e-5
    assert qsd["transformer.layers.0.input_layernorm.weight"].dtype == torch.float32


def test_quantized_split_scales(tmp_path):
    sd = _global_sd()
    files = _write(tmp_path, sd, 1, 2.0)
    loader = SDLoaderFactory.get_sd_loader(files, None, "Megatron", 2.0)
    _, got, (scales, _) = loader.load(2, 1, quantize=True, quantize_bits=8, quantize_groups=2)
    assert got["module"]["transformer.layers.0.attention.dense.weight"].dtype == torch.int8
    assert len(scales) == 2 and scales[1].shape[:2] == (L, 4)


def test_mp_world_size_mismatch_rejected(tmp_path):
    files = _write(tmp_path, _global_sd(), 2, 0)
    with pytest.raises(ValueError):
        MegatronSDLoader(files[:1], 0, None)


def test_init_inference_ds_model_descriptor(tmp_path):
    """HF-layout shards listed in a ds_model JSON stream into a meta-device model before injection."""
    transformers = pytest.importorskip("transformers")
    import deepspeedsyclsupport_amd as ds
    cfg = transformers.GPT2Config(n_layer=2, n_embd=32, n_head=4, vocab_size=64, n_positions=32)
    torch.manual_seed(0)
    src = transformers.GPT2LMHeadModel(cfg).eval()
    full = src.state_dict()
    keys = list(full.keys())
    shards = [dict((k, full[k]) for k in keys[:len(keys) // 2]), dict((k, full[k]) for k in keys[len(keys) // 2:])]
    names = []
    for i, s in enumerate(shards):
        torch.save(s, tmp_path / f"shard{i}.pt")
        names.append(f"shard{i}.pt")
    desc = tmp_path / "ckpt.json"
    desc.write_text(json.dumps({"type": "ds_model", "checkpoints": names, "version": 1.0}))
    with torch.device("meta"):
        model = transformers.GPT2LMHeadModel(cfg)
    eng = ds.init_inference(model, dtype=torch.float32, checkpoint=str(desc), base_dir=str(tmp_path),
                            replace_with_kernel_inject=False)
    ids = torch.randint(0, 64, (1, 8))
    with torch.no_grad():
        torch.testing.assert_close(eng.module(ids).logits, src(ids).logits, rtol=1e-5, atol=1e-5)
