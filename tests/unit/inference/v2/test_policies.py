"""Checkpoint directory -> ragged engine through the policy / container / checkpoint-engine path
(`inference/v2/{checkpoint,model_implementations}`; reference `engine_factory.py:65-129`,
`inference_policy_base.py`, `layer_container_base.py`): tiny random HF models are saved with `save_pretrained`, built
with `build_hf_engine(directory)` (streamed tensor by tensor, never instantiated as an HF model), and their logits
compared with the HF model."""
import pytest
import torch

from deepspeedsyclsupport_amd.inference.v2 import RaggedInferenceEngineConfig, build_hf_engine
from deepspeedsyclsupport_amd.inference.v2.checkpoint import HuggingFaceCheckpointEngine, InMemoryModelEngine
from deepspeedsyclsupport_amd.inference.v2.model_implementations import (POLICIES, ContainerMap, LayerContainer,
                                                                         ParameterBase, ParamList)
from deepspeedsyclsupport_amd.inference.v2.model_implementations import sharding
from deepspeedsyclsupport_amd.inference.v2.model_implementations.common_parameters import (
    GQAMegatronQKVParameter, MegatronQKVParameter, NormParameter, UnfusedQKVParameter)

from ..test_inference import tiny


def _cfg():
    return RaggedInferenceEngineConfig(state_manager={"max_context": 128, "max_ragged_batch_size": 128,
                                                      "max_ragged_sequence_count": 8,
                                                      "memory_config": {"mode": "allocate", "size": 32}})


@pytest.mark.parametrize("kind", ["llama", "mistral", "mixtral", "opt", "phi", "falcon", "falcon_new"])
@pytest.mark.parametrize("fmt", ["safetensors", "bin"])
def test_build_from_checkpoint_directory(kind, fmt, tmp_path, monkeypatch):
    if fmt == "bin" and kind != "llama":
        pytest.skip("the .bin reader is format-, not architecture-specific")
    m = tiny(kind).eval()
    assert m.config.model_type in POLICIES
    m.save_pretrained(str(tmp_path), safe_serialization=(fmt == "safetensors"))
    import transformers
    monkeypatch.setattr(transformers.AutoModelForCausalLM, "from_pretrained",
                        lambda *a, **k: pytest.fail("the policy path must not instantiate the HF model"))
    eng = build_hf_engine(str(tmp_path), _cfg(), dtype=torch.float32)
    ids = torch.randint(0, m.config.vocab_size, (2, 11), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = m(ids).logits[:, -1]
    out = eng.put([1, 2], [ids[0], ids[1]])
    torch.testing.assert_close(out, ref, rtol=2e-4, atol=2e-4)


def test_checkpoint_engines(tmp_path):
    m = tiny("llama")
    m.save_pretrained(str(tmp_path), safe_serialization=True)
    eng = HuggingFaceCheckpointEngine(str(tmp_path))
    assert eng.model_config.model_type == "llama"
    got = dict(eng.parameters())
    sd = m.state_dict()
    assert set(got) <= set(sd) and len(got) >= len(sd) - 1      # a tied lm_head may be stored once
    torch.testing.assert_close(got["model.layers.1.mlp.up_proj.weight"], sd["model.layers.1.mlp.up_proj.weight"])
    mem = dict(InMemoryModelEngine(m).parameters())
    assert set(mem) <= set(sd) and "model.embed_tokens.weight" in mem
    with pytest.raises(FileNotFoundError):
        HuggingFaceCheckpointEngine(str(tmp_path / "nope"))


def test_container_rules():
    class View:
        n_experts = 3

        class spec:
            num_heads, num_kv_heads, head_dim = 4, 2, 8

    class Experts(ParameterBase):
        experts: ParamList("n_experts")

        def finalize(self):
            return {"stack": torch.stack(list(self.experts))}

    class C(LayerContainer):
        qkv: UnfusedQKVParameter
        norm: NormParameter.as_("ln1_w")
        moe: Experts
        PARAM_MAPPING = {"attn.q.weight": "qkv.q_params", "attn.k.weight": "qkv.k_params",
                         "attn.v.weight": "qkv.v_params", "*ln.weight": ["norm.params"],
                         "experts.*.w": "moe.experts"}

    c = C(View)
    assert not c.is_initialized
    for n in ("q", "k"):
        assert c.set_dependency(f"attn.{n}.weight", torch.ones(2))
    assert not c.is_initialized and c.missing() == ["qkv.v_params"]
    c.set_dependency("attn.v.weight", torch.ones(2))
    c.set_dependency("some.prefix.ln.weight", torch.zeros(2))
    for i in range(3):
        c.set_dependency(f"experts.{i}.w", torch.full((2, ), float(i)))
    assert c.is_initialized and not c.set_dependency("unknown", torch.ones(1))
    out = c.canonical()
    assert set(out) == {"q_w", "k_w", "v_w", "ln1_w", "stack"} and out["stack"][:, 0].tolist() == [0.0, 1.0, 2.0]
    with pytest.raises(ValueError, match="names no annotated parameter"):
        type("Bad", (LayerContainer, ), {"PARAM_MAPPING": {"a": "nope.params"}})(View)

    # fused layouts
    D, nh, nk = 8, 4, 2
    q, k, v = torch.randn(nh * D, 5), torch.randn(nk * D, 5), torch.randn(nk * D, 5)
    p = MegatronQKVParameter(View)
    inter = torch.stack([q.view(nh, D, 5), torch.randn(nh, D, 5), torch.randn(nh, D, 5)], 1).reshape(-1, 5)
    p.set_field("params", inter)
    torch.testing.assert_close(p.finalize()["q_w"], q)
    g = GQAMegatronQKVParameter(View)
    grouped = torch.cat([torch.cat([q.view(nk, 2 * D, 5)[i], k.view(nk, D, 5)[i], v.view(nk, D, 5)[i]])
                         for i in range(nk)])
    g.set_field("params", grouped)
    fin = g.finalize()
    torch.testing.assert_close(fin["q_w"], q)
    torch.testing.assert_close(fin["v_w"], v)

    cm = ContainerMap()
    cm.set_transformer_params("m.layers", [C(View), C(View)])
    cm.set_non_transformer_params(C(View))
    cm.set_unmapped_params([r"inv_freq$"])
    assert cm.map_param("m.layers.1.attn.q.weight", torch.ones(2)) == 1
    assert cm.map_param("m.layers.0.rotary.inv_freq", torch.ones(2)) == 0
    with pytest.raises(ValueError, match="Cannot find container"):
        cm.map_param("m.layers.0.bogus", torch.ones(2))
    with pytest.raises(RuntimeError, match="not fully initialized"):
        cm.validate()


def test_sharding_rules():
    D, nq, nkv = 4, 8, 2
    qkv = torch.arange((nq + 2 * nkv) * D).float()[:, None].repeat(1, 3)
    parts = [sharding.shard_qkv_param(qkv, r, 4, D, nq, nkv) for r in range(4)]
    assert all(p.shape[0] == sharding.qkv_out_features(nq * D, r, 4, D, nq, nkv) == (2 + 2) * D
               for r, p in enumerate(parts))
    # ranks 0, 1 share kv head 0; ranks 2, 3 share kv head 1
    k0 = qkv[nq * D:nq * D + D]
    torch.testing.assert_close(parts[0][2 * D:3 * D], k0)
    torch.testing.assert_close(parts[1][2 * D:3 * D], k0)
    torch.testing.assert_close(parts[3][2 * D:3 * D], qkv[nq * D + D:nq * D + 2 * D])
    assert sharding.get_local_heads(1, 4, nq, nkv) == (2, 1) and sharding.get_local_heads(0, 2, nq, nkv) == (4, 1)
    o = torch.randn(16, nq * D)
    torch.testing.assert_close(torch.cat([sharding.shard_attn_out_param(o, r, 4, D, nq, nkv) for r in range(4)], 1), o)
    assert sharding.shard_attn_out_param(torch.ones(16), 1, 4, D) is None
    # uneven intermediate: 5 granules over 2 ranks -> 3 + 2
    assert [sharding.sharded_intermediate_dim(160, 2, r) for r in range(2)] == [96, 64]
    gate_up = torch.randn(2 * 160, 8)
    s0 = sharding.shard_mlp_1_param(gate_up, 0, 2, gated=True)
    torch.testing.assert_close(s0, torch.cat([gate_up[:96], gate_up[160:256]]))
    down = torch.randn(8, 160)
    torch.testing.assert_close(torch.cat([sharding.shard_mlp_2_param(down, r, 2) for r in range(2)], 1), down)
    assert sharding.sharded_unembed_dim(101, 0, 2) + sharding.sharded_unembed_dim(101, 1, 2) == 101
    with pytest.raises(ValueError):
        sharding.get_shard_endpoints(100, 0, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["llama", "mixtral", "falcon"])
def test_build_from_checkpoint_directory_gpu(kind, tmp_path):
    """The streamed policy load into the bf16 device model, prompt + one decode step through the HIP kernels."""
    m = tiny(kind, H=256).eval()
    m.save_pretrained(str(tmp_path), safe_serialization=True)
    eng = build_hf_engine(str(tmp_path), _cfg(), dtype=torch.bfloat16)
    assert eng.model.layers[0].qkv_w.is_cuda and eng.model.dtype == torch.bfloat16
    ids = torch.randint(0, m.config.vocab_size, (2, 21), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref_prompt = m(ids[:, :20]).logits[:, -1].float()
        ref_next = m(ids).logits[:, -1].float()
    out = eng.put([1, 2], [ids[0, :20], ids[1, :20]]).float().cpu()
    assert (out - ref_prompt).abs().max().item() < 0.05 * ref_prompt.abs().max().item() + 0.02
    out = eng.put([1, 2], [ids[0, 20:], ids[1, 20:]]).float().cpu()
    assert (out - ref_next).abs().max().item() < 0.05 * ref_next.abs().max().item() + 0.02
