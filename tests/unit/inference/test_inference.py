"""Kernel-injected inference (reference `tests/unit/inference/test_inference.py`: per-model output parity of
`init_inference` against the HF pipeline, TP via `mp_size`, int8 quantisation, CUDA graphs).

HF reference models are tiny random-init instances built from their configs (no network / checkpoints). CPU runs
use fp32 and demand near-bitwise parity; TP=2 runs use gloo ranks; GPU tests check the bf16 HIP path (paged decode,
fused kernels, HIP-graph decode) against the fp32 HF model.
"""
import pytest
import torch

from ..common import run_distributed

transformers = pytest.importorskip("transformers")
V = 256


def tiny(kind, H=64):
    """Tiny random model; 4 heads so head_dim = H / 4 (GPU tests use H=256 -> D=64, the decode kernel path)."""
    T = transformers
    torch.manual_seed(0)
    if kind == "llama":
        c = T.LlamaConfig(vocab_size=V, hidden_size=H, intermediate_size=2 * H, num_hidden_layers=2,
                          num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
        return T.LlamaForCausalLM(c)
    if kind == "mistral":
        c = T.MistralConfig(vocab_size=V, hidden_size=H, intermediate_size=2 * H, num_hidden_layers=2,
                            num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128,
                            sliding_window=8)
        return T.MistralForCausalLM(c)
    if kind == "qwen2":
        c = T.Qwen2Config(vocab_size=V, hidden_size=H, intermediate_size=2 * H, num_hidden_layers=2,
                          num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
        return T.Qwen2ForCausalLM(c)
    if kind == "gpt_neo":
        return T.GPTNeoForCausalLM(T.GPTNeoConfig(vocab_size=V, hidden_size=H, num_layers=4, num_heads=4,
                                                  attention_types=[[["global", "local"], 2]], window_size=5,
                                                  max_position_embeddings=128, bos_token_id=0, eos_token_id=1))
    if kind == "gpt2":
        return T.GPT2LMHeadModel(T.GPT2Config(vocab_size=V, n_embd=H, n_layer=2, n_head=4, n_positions=128,
                                              bos_token_id=0, eos_token_id=1))
    if kind == "bloom":
        return T.BloomForCausalLM(T.BloomConfig(vocab_size=V, hidden_size=H, n_layer=2, n_head=4))
    if kind == "opt":
        return T.OPTForCausalLM(T.OPTConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2, ffn_dim=2 * H,
                                            num_attention_heads=4, max_position_embeddings=128,
                                            word_embed_proj_dim=H))
    if kind == "gpt_neox":
        return T.GPTNeoXForCausalLM(T.GPTNeoXConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2,
                                                    num_attention_heads=4, intermediate_size=2 * H,
                                                    max_position_embeddings=128))
    if kind == "gptj":
        return T.GPTJForCausalLM(T.GPTJConfig(vocab_size=V, n_embd=H, n_layer=2, n_head=4, rotary_dim=8,
                                              n_positions=128, bos_token_id=0, eos_token_id=1))
    if kind == "mixtral":
        c = T.MixtralConfig(vocab_size=V, hidden_size=H, intermediate_size=2 * H, num_hidden_layers=2,
                            num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128,
                            num_local_experts=4, num_experts_per_tok=2)
        return T.MixtralForCausalLM(c)
    if kind in ("falcon", "falcon_new", "falcon_seq"):
        kw = dict(vocab_size=V, hidden_size=H, num_hidden_layers=2, num_attention_heads=4,
                  max_position_embeddings=128, bos_token_id=0, eos_token_id=1)
        if kind == "falcon_new":  # 40B/180B layout: grouped kv heads, ln_attn + ln_mlp
            kw.update(new_decoder_architecture=True, num_kv_heads=2)
        if kind == "falcon_seq":  # sequential residual, full MHA with interleaved qkv, biased linears
            kw.update(parallel_attn=False, multi_query=False, bias=True)
        return T.FalconForCausalLM(T.FalconConfig(**kw))
    if kind == "phi":
        return T.PhiForCausalLM(T.PhiConfig(vocab_size=V, hidden_size=H, intermediate_size=2 * H,
                                            num_hidden_layers=2, num_attention_heads=4, max_position_embeddings=128,
                                            partial_rotary_factor=0.5, bos_token_id=0, eos_token_id=1))
    raise ValueError(kind)


ARCHS = ["llama", "mistral", "qwen2", "gpt2", "bloom", "opt", "gpt_neox", "gptj", "mixtral", "falcon", "falcon_new",
         "falcon_seq", "phi", "gpt_neo"]


def _ids(B=2, S=12, seed=1):
    return torch.randint(2, V, (B, S), generator=torch.Generator().manual_seed(seed))


@pytest.mark.parametrize("kind", ARCHS)
def test_injected_parity_cpu(kind):
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind).eval()
    ids = _ids()
    with torch.no_grad():
        ref = m(ids).logits
    eng = ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=True)
    assert eng.injected
    out = eng(ids).logits
    assert (out - ref).abs().max().item() < 1e-4
    g_ref = m.generate(ids, max_new_tokens=6, do_sample=False, pad_token_id=0)
    assert torch.equal(eng.generate(ids, max_new_tokens=6), g_ref)


def test_padded_batch_and_sampling():
    import deepspeedsyclsupport_amd as ds
    m = tiny("llama").eval()
    ids = _ids()
    mask = torch.ones_like(ids)
    ids[0, :4], mask[0, :4] = 0, 0
    eng = ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=True)
    g = eng.generate(ids, attention_mask=mask, max_new_tokens=5)
    assert torch.equal(g[0, -5:], m.generate(ids[0:1, 4:], max_new_tokens=5, do_sample=False)[0, -5:])
    assert torch.equal(g[1], m.generate(ids[1:2], max_new_tokens=5, do_sample=False)[0])
    s1 = eng.generate(ids[1:], max_new_tokens=5, do_sample=True, top_k=10, top_p=0.9, temperature=0.8, seed=3)
    s2 = eng.generate(ids[1:], max_new_tokens=5, do_sample=True, top_k=10, top_p=0.9, temperature=0.8, seed=3)
    assert torch.equal(s1, s2) and s1.shape == (1, 17)


def test_eos_stops_and_pads():
    import deepspeedsyclsupport_amd as ds
    m = tiny("llama").eval()
    ids = _ids(B=1)
    eng = ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=True)
    g = eng.generate(ids, max_new_tokens=8)
    eos = int(g[0, 14])  # force the third generated token to be "EOS"
    g2 = eng.generate(ids, max_new_tokens=8, eos_token_id=eos, pad_token_id=0)
    assert int(g2[0, 14]) == eos and (g2[0, 15:] == 0).all()


def test_int8_weight_quant():
    import deepspeedsyclsupport_amd as ds
    m = tiny("llama").eval()
    ids = _ids(B=1)
    with torch.no_grad():
        ref = m(ids).logits
    eng = ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=True,
                            quant={"enabled": True, "weight": {"num_bits": 8}})
    err = (eng(ids).logits - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item()


def test_native_llama_injection():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.models.llama import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig(vocab_size=V, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                     num_attention_heads=4, num_key_value_heads=2)).eval()
    ids = _ids()
    with torch.no_grad():
        ref = m(ids)
    ref = ref.logits if hasattr(ref, "logits") else ref
    eng = ds.init_inference(m, dtype=torch.float32)
    assert eng.injected
    assert (eng(ids).logits - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("kind", ["llama", "gpt2", "bloom"])
def test_revert_transformer_layer_round_trip(kind):
    """replace -> edit the injected weights -> revert: the original module comes back carrying the edit (reference
    `module_inject/replace_module.py` revert_transformer_layer)."""
    from deepspeedsyclsupport_amd.inference.config import DeepSpeedInferenceConfig
    from deepspeedsyclsupport_amd.module_inject import replace_transformer_layer, revert_transformer_layer
    m = tiny(kind).eval()
    ids = _ids()
    cfg = DeepSpeedInferenceConfig(dtype="fp32")
    inj = replace_transformer_layer(None, m, config=cfg)
    with torch.no_grad():
        ref = m(ids).logits.clone()
        back = revert_transformer_layer(None, inj, cfg)
        assert back is m
        assert (m(ids).logits - ref).abs().max().item() < 1e-5  # an unedited round trip changes nothing
        for layer in inj.layers:
            layer.o_w.mul_(0.5)
            layer.fc2_w.mul_(2.0)
        revert_transformer_layer(None, inj, cfg)
        from deepspeedsyclsupport_amd.inference.model_implementations import convert
        _, _, lws = convert.extract(m)
        for lw, layer in zip(lws, inj.layers):
            torch.testing.assert_close(lw["o_w"].contiguous(), layer.o_w.data, rtol=0, atol=0)
            if "fc2_w" in lw:
                torch.testing.assert_close(lw["fc2_w"].contiguous(), layer.fc2_w.data, rtol=0, atol=0)
        assert (m(ids).logits - ref).abs().max().item() > 1e-4  # and the original model now computes with them
    with pytest.raises(ValueError):
        revert_transformer_layer(None, torch.nn.Linear(2, 2), cfg)


def test_config_aliases():
    from deepspeedsyclsupport_amd.inference.config import DeepSpeedInferenceConfig
    c = DeepSpeedInferenceConfig(kernel_inject=True, dtype="bf16", mp_size=2, max_tokens=77)
    assert c.replace_with_kernel_inject and c.dtype == torch.bfloat16
    assert c.tensor_parallel.tp_size == 2 and c.max_out_tokens == 77
    with pytest.raises(Exception):
        DeepSpeedInferenceConfig(not_a_key=1)


# ---------------------------------------------------------------------------------------------- tensor parallel
def _tp_run(kind, inject):
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind).eval()
    ids = _ids()
    with torch.no_grad():
        ref = m(ids).logits
    g_ref = m.generate(ids, max_new_tokens=4, do_sample=False, pad_token_id=0) if inject else None
    eng = ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=inject,
                            tensor_parallel={"tp_size": 2})
    out = eng(ids)
    out = out.logits if hasattr(out, "logits") else out[0]
    err = (out - ref).abs().max().item()
    assert err < 1e-4, f"{kind} inject={inject} tp2 err {err}"
    if inject:
        assert torch.equal(eng.generate(ids, max_new_tokens=4), g_ref)


@pytest.mark.parametrize("kind", ["llama", "bloom", "gpt2", "mixtral", "falcon", "falcon_new", "phi", "gpt_neo"])
def test_tp2_injected(kind):
    run_distributed(_tp_run, 2, kind, True)


@pytest.mark.parametrize("kind", ["llama", "gpt2", "opt"])
def test_tp2_autotp(kind):
    run_distributed(_tp_run, 2, kind, False)


# ---------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["llama", "bloom", "gpt_neox", "mixtral", "falcon", "phi", "gpt_neo"])
def test_injected_bf16_gpu(kind):
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind, H=256).eval()
    ids = _ids(B=3, S=20)
    with torch.no_grad():
        ref = m(ids).logits.float()
    eng = ds.init_inference(m, dtype=torch.bfloat16, replace_with_kernel_inject=True)
    out = eng(ids.cuda()).logits.float().cpu()
    assert (out - ref).abs().max().item() < 0.05 * ref.abs().max().item() + 0.02
    # decode through the paged HIP kernel: teacher-force the HF prompt+continuation and compare last-token logits
    g = eng.generate(ids.cuda(), max_new_tokens=8).cpu()
    with torch.no_grad():
        full = m(g[:, :-1]).logits[:, -1].float()
    step_logits = eng(g[:, :-1].cuda()).logits[:, -1].float().cpu()
    assert (step_logits - full).abs().max().item() < 0.05 * full.abs().max().item() + 0.02


@pytest.mark.gpu
@pytest.mark.parametrize("kind,H,D", [("gptj", 1024, 256), ("gpt_neox", 384, 96), ("phi", 320, 80), ("gpt2", 256, 64)])
def test_head_dims_take_the_paged_kernels_gpu(kind, H, D, monkeypatch):
    """GPT-J (head dim 256), GPT-NeoX-20B (96) and Phi (80) shapes: prompt and decode attention run in the paged HIP
    kernels (reference `softmax_context` is head-size generic, `pt_binding.cpp:434-557`) — the per-sequence SDPA
    paths must not be reached — and match the fp32 HF model."""
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.inference.model_implementations import transformer as tr
    for name in ("_cached_attention", "_prefill_attention", "_seq_cached_attention"):
        monkeypatch.setattr(tr, name, lambda *a, _n=name, **k: pytest.fail(f"{_n} reached for head dim {D}"))
    m = tiny(kind, H=H).eval()
    assert H // 4 == D
    ids = _ids(B=3, S=100)
    with torch.no_grad():
        ref = m(ids).logits.float()
    eng = ds.init_inference(m, dtype=torch.bfloat16, replace_with_kernel_inject=True)
    out = eng(ids.cuda()).logits.float().cpu()
    assert (out - ref).abs().max().item() < 0.05 * ref.abs().max().item() + 0.02
    g = eng.generate(ids.cuda(), max_new_tokens=8).cpu()
    with torch.no_grad():
        full = m(g[:, :-1]).logits[:, -1].float()
    step_logits = eng(g[:, :-1].cuda()).logits[:, -1].float().cpu()
    assert (step_logits - full).abs().max().item() < 0.05 * full.abs().max().item() + 0.02


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["llama", "mixtral"])
def test_decode_graph_matches_eager_gpu(kind):
    """HIP-graph decode == eager decode. For Mixtral this also proves the MoE block is capturable: routing, expert
    offsets and the grouped GEMM's tile map all stay on the device (no host sync inside the step)."""
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind, H=256).eval()
    ids = _ids(B=4, S=16).cuda()
    e1 = ds.init_inference(m, dtype=torch.bfloat16, replace_with_kernel_inject=True)
    e2 = ds.init_inference(m, dtype=torch.bfloat16, replace_with_kernel_inject=True, enable_cuda_graph=True)
    a = e1.generate(ids, max_new_tokens=12)
    b = e2.generate(ids, max_new_tokens=12)
    assert e2.cuda_graph_created
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["llama", "bloom"])
def test_int8_decode_gpu(kind):
    """Weight-only int8 on the GPU: decode steps (<= 8 rows) take the fused-dequant skinny kernel, prefill the
    dequantise + GEMM path; greedy tokens and last-token logits must follow the bf16 engine."""
    import copy

    import deepspeedsyclsupport_amd as ds
    m = tiny(kind, H=256).eval()
    ids = _ids(B=2, S=12).cuda()
    e16 = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True)
    e8 = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True,
                           quant={"enabled": True, "weight": {"num_bits": 8}})
    assert e8.module.layers[0].quant, "weights were not quantised"
    g16 = e16.generate(ids, max_new_tokens=6)
    l16 = e16(g16[:, :-1]).logits[:, -1].float()
    l8 = e8(g16[:, :-1]).logits[:, -1].float()
    assert (l8 - l16).abs().max().item() < 0.05 * l16.abs().max().item() + 0.05
    g8 = e8.generate(ids, max_new_tokens=6)
    assert g8.shape == g16.shape


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["both", "shuffled", "auto"])
@pytest.mark.parametrize("B", [1, 4, 16])
def test_bf16_decode_layouts_gpu(layout, B):
    """`decode_layout`: batched decode over the shuffled bf16 copies (2 - 16 token rows; "shuffled": every decode
    step, prefill un-shuffling per GEMM) must follow the row-major engine — same greedy tokens, close logits — with
    and without HIP graphs, and the layouts are really in place."""
    import copy

    import deepspeedsyclsupport_amd as ds
    m = tiny("llama", H=256).eval()
    ids = _ids(B=B, S=20).cuda()  # (prompts longer than 16 rows: prefill never takes the decode streams)
    ref = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True,
                            decode_layout="row_major")
    eng = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True,
                            decode_layout=layout)
    engg = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True,
                             decode_layout=layout, enable_cuda_graph=True)
    l0 = eng.module.layers[0]
    assert not ref.module.layers[0].sh and not ref.module.layers[0].quant
    if layout == "shuffled":
        assert l0.quant and l0.qkv_w.numel() == 0
    else:
        assert l0.sh and l0.qkv_w.numel() > 0
    g0 = ref.generate(ids, max_new_tokens=8)
    lr = ref(g0[:, :-1]).logits[:, -1].float()
    le = eng(g0[:, :-1]).logits[:, -1].float()
    assert (le - lr).abs().max().item() < 0.03 * lr.abs().max().item() + 0.03
    # one decode step from the same cache state, through the stream that this batch size selects
    from deepspeedsyclsupport_amd.ops import bf16_gemv
    calls = {"raw": 0}
    orig = bf16_gemv.Bf16Weight.raw

    def spy(self, x, bias=None):
        calls["raw"] += 1
        return orig(self, x, bias)

    bf16_gemv.Bf16Weight.raw = spy
    try:
        g1 = eng.generate(ids, max_new_tokens=8)
    finally:
        bf16_gemv.Bf16Weight.raw = orig
    expect_stream = layout == "shuffled" or B >= l0.SH_MIN_ROWS
    assert (calls["raw"] > 0) == expect_stream
    g2 = engg.generate(ids, max_new_tokens=8)
    assert torch.equal(g1, g2)
    # greedy decoding may legitimately diverge after a near-tie; the first new token comes from the prefill logits
    assert torch.equal(g1[:, :21], g0[:, :21]) or (le - lr).abs().max().item() < 0.05
