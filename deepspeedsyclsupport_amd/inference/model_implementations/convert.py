"""HF / native checkpoints -> `DSInferenceModel` (reference injection policies `module_inject/containers/*.py`
(llama, gpt2, bloom, opt, gptneox, gptj, ...) and v2 `model_implementations/*/policy.py` + `checkpoint/`).

Each converter maps a source model to a `DSModelSpec` plus per-layer CANONICAL full weights
(q/k/v/o, gate/up or fc1, fc2, norms, biases). `load_into` then shards them for tensor parallelism:
  q rows by heads, k/v rows by kv heads (replicated when kv_heads < tp), o columns by heads,
  gate/up/fc1 rows by intermediate, fc2 columns by intermediate, lm_head rows by vocab (zero-padded).
Fused/interleaved source layouts are untangled here: BLOOM/GPT-NeoX qkv is [heads, 3, D] interleaved, GPT-2 uses
Conv1D ([in, out]) weights, OPT learned positions have an offset of 2.
"""
import torch

from .transformer import DSInferenceModel, DSModelSpec


def _rope(cfg, default_theta=10000.0):
    rp = getattr(cfg, "rope_parameters", None) or getattr(cfg, "rope_scaling", None) or {}
    theta = rp.get("rope_theta", None) if isinstance(rp, dict) else None
    if theta is None:
        theta = getattr(cfg, "rope_theta", None) or getattr(cfg, "rotary_emb_base", None) or default_theta
    partial = rp.get("partial_rotary_factor", None) if isinstance(rp, dict) else None
    if partial is None:
        partial = getattr(cfg, "partial_rotary_factor", None) or getattr(cfg, "rotary_pct", None) or 1.0
    return float(theta), float(partial)


def _t(x):
    return None if x is None else x.detach()


# ------------------------------------------------------------------------------------------------ converters
def _llama_like(model):
    cfg = model.config
    theta, partial = _rope(cfg)
    nh = cfg.num_attention_heads
    hd = getattr(cfg, "head_dim", None) or cfg.hidden_size // nh
    spec = DSModelSpec(arch=cfg.model_type, vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                       num_layers=cfg.num_hidden_layers, num_heads=nh,
                       num_kv_heads=getattr(cfg, "num_key_value_heads", None) or nh,
                       intermediate_size=cfg.intermediate_size, head_dim=hd, norm="rms", norm_eps=cfg.rms_norm_eps,
                       pos="rope", rope_theta=theta, rotary_dim=int(hd * partial), act=cfg.hidden_act,
                       gated_mlp=True, qkv_bias=bool(getattr(cfg, "attention_bias", False)) or cfg.model_type == "qwen2",
                       o_bias=False, max_positions=cfg.max_position_embeddings,
                       sliding_window=(getattr(cfg, "sliding_window", None) or 0)
                       if getattr(cfg, "use_sliding_window", True) else 0,
                       tie_embeddings=bool(getattr(cfg, "tie_word_embeddings", False)))
    base = model.model
    layers = []
    for L in base.layers:
        a, m = L.self_attn, L.mlp
        layers.append(dict(ln1_w=L.input_layernorm.weight, ln2_w=L.post_attention_layernorm.weight,
                           q_w=a.q_proj.weight, k_w=a.k_proj.weight, v_w=a.v_proj.weight,
                           q_b=_t(a.q_proj.bias), k_b=_t(a.k_proj.bias), v_b=_t(a.v_proj.bias),
                           o_w=a.o_proj.weight, o_b=_t(a.o_proj.bias),
                           gate_w=m.gate_proj.weight, up_w=m.up_proj.weight, fc2_w=m.down_proj.weight))
    top = dict(embed=base.embed_tokens.weight, norm_w=base.norm.weight, lm_head=model.lm_head.weight)
    return spec, top, layers


def _native_llama(model):
    """Our own training `models.llama.LlamaForCausalLM` (fused qkv_proj / gate_up_proj)."""
    cfg = model.config
    nh, nk = cfg.num_attention_heads, cfg.num_key_value_heads or cfg.num_attention_heads
    hd = cfg.hidden_size // nh
    spec = DSModelSpec(arch="llama", vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                       num_layers=cfg.num_hidden_layers, num_heads=nh, num_kv_heads=nk,
                       intermediate_size=cfg.intermediate_size, norm="rms", norm_eps=cfg.rms_norm_eps, pos="rope",
                       rope_theta=cfg.rope_theta, act=cfg.hidden_act, gated_mlp=True,
                       qkv_bias=bool(cfg.attention_bias), max_positions=cfg.max_position_embeddings)
    base = model.model
    layers = []
    I = cfg.intermediate_size
    for L in base.layers:
        a, m = L.self_attn, L.mlp
        q, k, v = a.qkv_proj.weight.split([nh * hd, nk * hd, nk * hd], 0)
        qb = kb = vb = None
        if a.qkv_proj.bias is not None:
            qb, kb, vb = a.qkv_proj.bias.split([nh * hd, nk * hd, nk * hd], 0)
        layers.append(dict(ln1_w=L.input_layernorm.weight, ln2_w=L.post_attention_layernorm.weight, q_w=q, k_w=k,
                           v_w=v, q_b=qb, k_b=kb, v_b=vb, o_w=a.o_proj.weight, gate_w=m.gate_up_proj.weight[:I],
                           up_w=m.gate_up_proj.weight[I:], fc2_w=m.down_proj.weight))
    top = dict(embed=base.embed_tokens.weight, norm_w=base.norm.weight, lm_head=model.lm_head.weight)
    return spec, top, layers


def _split_interleaved(w, nh, hd):
    """[nh*3*D, ...] laid out [nh, 3, D] -> q, k, v each [nh*D, ...]."""
    shp = w.shape[1:]
    w = w.reshape(nh, 3, hd, *shp)
    return [w[:, i].reshape(nh * hd, *shp) for i in range(3)]


def _gpt2(model):
    cfg = model.config
    H, nh = cfg.n_embd, cfg.n_head
    spec = DSModelSpec(arch="gpt2", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.n_layer, num_heads=nh,
                       num_kv_heads=nh, intermediate_size=cfg.n_inner or 4 * H, norm="ln",
                       norm_eps=cfg.layer_norm_epsilon, pos="learned", act=cfg.activation_function, gated_mlp=False,
                       qkv_bias=True, o_bias=True, mlp_bias=True, max_positions=cfg.n_positions, tie_embeddings=True)
    tr = model.transformer
    layers = []
    for L in tr.h:
        at, mlp = L.attn, L.mlp
        wqkv = at.c_attn.weight.t()  # Conv1D stores [in, out]
        q, k, v = wqkv.split(H, 0)
        qb, kb, vb = at.c_attn.bias.split(H, 0)
        layers.append(dict(ln1_w=L.ln_1.weight, ln1_b=L.ln_1.bias, ln2_w=L.ln_2.weight, ln2_b=L.ln_2.bias, q_w=q,
                           k_w=k, v_w=v, q_b=qb, k_b=kb, v_b=vb, o_w=at.c_proj.weight.t(), o_b=at.c_proj.bias,
                           fc1_w=mlp.c_fc.weight.t(), fc1_b=mlp.c_fc.bias, fc2_w=mlp.c_proj.weight.t(),
                           fc2_b=mlp.c_proj.bias))
    top = dict(embed=tr.wte.weight, pos_embed=tr.wpe.weight, norm_w=tr.ln_f.weight, norm_b=tr.ln_f.bias,
               lm_head=model.lm_head.weight)
    return spec, top, layers


def _gpt_neo(model):
    """GPT-Neo (reference container `module_inject/containers/gptneo.py`): learned positions, un-scaled attention
    scores, alternating global / local (sliding-window) attention layers, biasless q/k/v."""
    cfg = model.config
    H, nh = cfg.hidden_size, cfg.num_heads
    windows = tuple(cfg.window_size if t == "local" else 0 for t in cfg.attention_layers)
    spec = DSModelSpec(arch="gpt_neo", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.num_layers,
                       num_heads=nh, num_kv_heads=nh, intermediate_size=cfg.intermediate_size or 4 * H, norm="ln",
                       norm_eps=cfg.layer_norm_epsilon, pos="learned", act=cfg.activation_function, gated_mlp=False,
                       qkv_bias=False, o_bias=True, mlp_bias=True, max_positions=cfg.max_position_embeddings,
                       tie_embeddings=True, layer_windows=windows, attn_scale=1.0)
    tr = model.transformer
    layers = []
    for L in tr.h:
        at, mlp = L.attn.attention, L.mlp
        layers.append(dict(ln1_w=L.ln_1.weight, ln1_b=L.ln_1.bias, ln2_w=L.ln_2.weight, ln2_b=L.ln_2.bias,
                           q_w=at.q_proj.weight, k_w=at.k_proj.weight, v_w=at.v_proj.weight,
                           o_w=at.out_proj.weight, o_b=at.out_proj.bias, fc1_w=mlp.c_fc.weight, fc1_b=mlp.c_fc.bias,
                           fc2_w=mlp.c_proj.weight, fc2_b=mlp.c_proj.bias))
    top = dict(embed=tr.wte.weight, pos_embed=tr.wpe.weight, norm_w=tr.ln_f.weight, norm_b=tr.ln_f.bias,
               lm_head=model.lm_head.weight)
    return spec, top, layers


def _bloom(model):
    cfg = model.config
    H, nh = cfg.hidden_size, cfg.n_head
    hd = H // nh
    spec = DSModelSpec(arch="bloom", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.n_layer, num_heads=nh,
                       num_kv_heads=nh, intermediate_size=4 * H, norm="ln", norm_eps=cfg.layer_norm_epsilon,
                       pos="alibi", act="gelu_tanh", gated_mlp=False, qkv_bias=True, o_bias=True, mlp_bias=True,
                       embed_norm=True, tie_embeddings=True, max_positions=2048)
    assert not cfg.apply_residual_connection_post_layernorm, "post-LN residual BLOOM variant unsupported"
    tr = model.transformer
    layers = []
    for L in tr.h:
        sa, mlp = L.self_attention, L.mlp
        q, k, v = _split_interleaved(sa.query_key_value.weight, nh, hd)
        qb, kb, vb = _split_interleaved(sa.query_key_value.bias, nh, hd)
        layers.append(dict(ln1_w=L.input_layernorm.weight, ln1_b=L.input_layernorm.bias,
                           ln2_w=L.post_attention_layernorm.weight, ln2_b=L.post_attention_layernorm.bias, q_w=q,
                           k_w=k, v_w=v, q_b=qb, k_b=kb, v_b=vb, o_w=sa.dense.weight, o_b=sa.dense.bias,
                           fc1_w=mlp.dense_h_to_4h.weight, fc1_b=mlp.dense_h_to_4h.bias,
                           fc2_w=mlp.dense_4h_to_h.weight, fc2_b=mlp.dense_4h_to_h.bias))
    top = dict(embed=tr.word_embeddings.weight, embed_ln_w=tr.word_embeddings_layernorm.weight,
               embed_ln_b=tr.word_embeddings_layernorm.bias, norm_w=tr.ln_f.weight, norm_b=tr.ln_f.bias,
               lm_head=model.lm_head.weight)
    return spec, top, layers


def _opt(model):
    cfg = model.config
    H, nh = cfg.hidden_size, cfg.num_attention_heads
    assert cfg.do_layer_norm_before and cfg.word_embed_proj_dim == H, "OPT-350m style projections unsupported"
    spec = DSModelSpec(arch="opt", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.num_hidden_layers,
                       num_heads=nh, num_kv_heads=nh, intermediate_size=cfg.ffn_dim, norm="ln", norm_eps=1e-5,
                       pos="learned", learned_pos_offset=2, act=cfg.activation_function, gated_mlp=False,
                       qkv_bias=cfg.enable_bias, o_bias=cfg.enable_bias, mlp_bias=cfg.enable_bias,
                       max_positions=cfg.max_position_embeddings, tie_embeddings=True)
    dec = model.model.decoder
    layers = []
    for L in dec.layers:
        a = L.self_attn
        layers.append(dict(ln1_w=L.self_attn_layer_norm.weight, ln1_b=L.self_attn_layer_norm.bias,
                           ln2_w=L.final_layer_norm.weight, ln2_b=L.final_layer_norm.bias, q_w=a.q_proj.weight,
                           k_w=a.k_proj.weight, v_w=a.v_proj.weight, q_b=_t(a.q_proj.bias), k_b=_t(a.k_proj.bias),
                           v_b=_t(a.v_proj.bias), o_w=a.out_proj.weight, o_b=_t(a.out_proj.bias), fc1_w=L.fc1.weight,
                           fc1_b=_t(L.fc1.bias), fc2_w=L.fc2.weight, fc2_b=_t(L.fc2.bias)))
    top = dict(embed=dec.embed_tokens.weight, pos_embed=dec.embed_positions.weight, norm_w=dec.final_layer_norm.weight,
               norm_b=dec.final_layer_norm.bias, lm_head=model.lm_head.weight)
    return spec, top, layers


def _gpt_neox(model):
    cfg = model.config
    H, nh = cfg.hidden_size, cfg.num_attention_heads
    hd = H // nh
    theta, partial = _rope(cfg)
    spec = DSModelSpec(arch="gpt_neox", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.num_hidden_layers,
                       num_heads=nh, num_kv_heads=nh, intermediate_size=cfg.intermediate_size, norm="ln",
                       norm_eps=cfg.layer_norm_eps, pos="rope", rope_theta=theta, rotary_dim=int(hd * partial),
                       act=cfg.hidden_act, gated_mlp=False, qkv_bias=True, o_bias=True, mlp_bias=True,
                       parallel_residual=cfg.use_parallel_residual, max_positions=cfg.max_position_embeddings)
    base = model.gpt_neox
    layers = []
    for L in base.layers:
        a, mlp = L.attention, L.mlp
        q, k, v = _split_interleaved(a.query_key_value.weight, nh, hd)
        qb, kb, vb = _split_interleaved(a.query_key_value.bias, nh, hd)
        layers.append(dict(ln1_w=L.input_layernorm.weight, ln1_b=L.input_layernorm.bias,
                           ln2_w=L.post_attention_layernorm.weight, ln2_b=L.post_attention_layernorm.bias, q_w=q,
                           k_w=k, v_w=v, q_b=qb, k_b=kb, v_b=vb, o_w=a.dense.weight, o_b=a.dense.bias,
                           fc1_w=mlp.dense_h_to_4h.weight, fc1_b=mlp.dense_h_to_4h.bias,
                           fc2_w=mlp.dense_4h_to_h.weight, fc2_b=mlp.dense_4h_to_h.bias))
    top = dict(embed=base.embed_in.weight, norm_w=base.final_layer_norm.weight, norm_b=base.final_layer_norm.bias,
               lm_head=(model.embed_out if hasattr(model, "embed_out") else model.lm_head).weight)
    return spec, top, layers


def _gptj(model):
    cfg = model.config
    H, nh = cfg.n_embd, cfg.n_head
    spec = DSModelSpec(arch="gptj", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.n_layer, num_heads=nh,
                       num_kv_heads=nh, intermediate_size=cfg.n_inner or 4 * H, norm="ln",
                       norm_eps=cfg.layer_norm_epsilon, pos="rope_gptj", rotary_dim=cfg.rotary_dim or H // nh,
                       act=cfg.activation_function, gated_mlp=False, mlp_bias=True, parallel_residual=True,
                       shared_parallel_norm=True, max_positions=cfg.n_positions, lm_head_bias=True)
    tr = model.transformer
    layers = []
    for L in tr.h:
        a, mlp = L.attn, L.mlp
        layers.append(dict(ln1_w=L.ln_1.weight, ln1_b=L.ln_1.bias, q_w=a.q_proj.weight, k_w=a.k_proj.weight,
                           v_w=a.v_proj.weight, o_w=a.out_proj.weight, fc1_w=mlp.fc_in.weight, fc1_b=mlp.fc_in.bias,
                           fc2_w=mlp.fc_out.weight, fc2_b=mlp.fc_out.bias))
    top = dict(embed=tr.wte.weight, norm_w=tr.ln_f.weight, norm_b=tr.ln_f.bias, lm_head=model.lm_head.weight,
               lm_head_b=model.lm_head.bias)
    return spec, top, layers


def _mixtral(model):
    """Mixtral / Qwen2-MoE style sparse MLP (reference v2 `model_implementations/mixtral/`): the llama attention
    stack plus a top-k router over gated experts; HF keeps the experts fused as `gate_up_proj` [E, 2I, H] and
    `down_proj` [E, H, I]."""
    cfg = model.config
    spec, top, _ = _llama_like_spec_only(model)
    spec.arch = "mixtral"
    spec.num_experts = cfg.num_local_experts
    spec.moe_top_k = cfg.num_experts_per_tok
    base = model.model
    layers = []
    for L in base.layers:
        a, m = L.self_attn, L.mlp
        ex = m.experts
        layers.append(dict(ln1_w=L.input_layernorm.weight, ln2_w=L.post_attention_layernorm.weight,
                           q_w=a.q_proj.weight, k_w=a.k_proj.weight, v_w=a.v_proj.weight, o_w=a.o_proj.weight,
                           router_w=m.gate.weight, experts_gate_up=ex.gate_up_proj, experts_down=ex.down_proj))
    return spec, top, layers


def _llama_like_spec_only(model):
    cfg = model.config
    theta, partial = _rope(cfg)
    nh = cfg.num_attention_heads
    hd = getattr(cfg, "head_dim", None) or cfg.hidden_size // nh
    spec = DSModelSpec(arch=cfg.model_type, vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                       num_layers=cfg.num_hidden_layers, num_heads=nh,
                       num_kv_heads=getattr(cfg, "num_key_value_heads", None) or nh,
                       intermediate_size=cfg.intermediate_size, head_dim=hd, norm="rms", norm_eps=cfg.rms_norm_eps,
                       pos="rope", rope_theta=theta, rotary_dim=int(hd * partial), act=cfg.hidden_act,
                       gated_mlp=True, max_positions=cfg.max_position_embeddings,
                       sliding_window=getattr(cfg, "sliding_window", None) or 0,
                       tie_embeddings=bool(getattr(cfg, "tie_word_embeddings", False)))
    top = dict(embed=model.model.embed_tokens.weight, norm_w=model.model.norm.weight, lm_head=model.lm_head.weight)
    return spec, top, None


def _falcon(model):
    """Falcon 7B/40B/180B (reference `module_inject/containers` has no Falcon policy; v2 `model_implementations/
    falcon/`): fused query_key_value in one of three layouts, parallel attention+MLP with one shared or two
    separate LayerNorms, multi-query / grouped KV heads, rotary positions, bias-free GELU MLP."""
    cfg = model.config
    H, nh = cfg.hidden_size, cfg.num_attention_heads
    hd = H // nh
    assert not cfg.alibi, "ALiBi Falcon variants are not supported by the injected kernels"
    new = bool(cfg.new_decoder_architecture)
    nk = cfg.num_kv_heads if new else (1 if cfg.multi_query else nh)
    n_ln = (cfg.num_ln_in_parallel_attn or 2) if new else 1
    assert cfg.parallel_attn or not new, "sequential attention with the new decoder layout is not a Falcon model"
    theta, _ = _rope(cfg)
    spec = DSModelSpec(arch="falcon", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.num_hidden_layers,
                       num_heads=nh, num_kv_heads=nk, intermediate_size=getattr(cfg, "ffn_hidden_size", None) or 4 * H,
                       norm="ln", norm_eps=cfg.layer_norm_epsilon, pos="rope", rope_theta=theta, act="gelu",
                       gated_mlp=False, qkv_bias=cfg.bias, o_bias=cfg.bias, mlp_bias=cfg.bias,
                       parallel_residual=bool(cfg.parallel_attn),
                       shared_parallel_norm=bool(cfg.parallel_attn) and n_ln == 1,
                       max_positions=cfg.max_position_embeddings,
                       tie_embeddings=bool(getattr(cfg, "tie_word_embeddings", True)))

    def split(w):
        if w is None:
            return None, None, None
        shp = w.shape[1:]
        if new:
            g = w.reshape(nk, nh // nk + 2, hd, *shp)
            return g[:, :-2].reshape(nh * hd, *shp), g[:, -2].reshape(nk * hd, *shp), g[:, -1].reshape(nk * hd, *shp)
        if cfg.multi_query:
            return w.split([nh * hd, hd, hd], 0)
        return _split_interleaved(w, nh, hd)

    tr = model.transformer
    layers = []
    for L in tr.h:
        sa, mlp = L.self_attention, L.mlp
        q, k, v = split(sa.query_key_value.weight)
        qb, kb, vb = split(_t(sa.query_key_value.bias))
        if n_ln == 2:
            n1, n2 = L.ln_attn, L.ln_mlp
        else:
            n1 = L.input_layernorm
            n2 = getattr(L, "post_attention_layernorm", None) if not cfg.parallel_attn else None
        lw = dict(ln1_w=n1.weight, ln1_b=n1.bias, q_w=q, k_w=k, v_w=v, q_b=qb, k_b=kb, v_b=vb,
                  o_w=sa.dense.weight, o_b=_t(sa.dense.bias), fc1_w=mlp.dense_h_to_4h.weight,
                  fc1_b=_t(mlp.dense_h_to_4h.bias), fc2_w=mlp.dense_4h_to_h.weight, fc2_b=_t(mlp.dense_4h_to_h.bias))
        if n2 is not None:
            lw.update(ln2_w=n2.weight, ln2_b=n2.bias)
        layers.append(lw)
    top = dict(embed=tr.word_embeddings.weight, norm_w=tr.ln_f.weight, norm_b=tr.ln_f.bias,
               lm_head=model.lm_head.weight)
    return spec, top, layers


def _phi(model):
    """Phi-1/1.5/2 (reference v2 `model_implementations/phi/`): GPT-J-like parallel block with one shared
    LayerNorm, partial rotary (NeoX half-split over the first rotary_dim lanes), biased q/k/v/dense/fc1/fc2,
    gelu_new, final LayerNorm and a biased LM head."""
    cfg = model.config
    H, nh = cfg.hidden_size, cfg.num_attention_heads
    hd = H // nh
    theta, partial = _rope(cfg)
    assert not getattr(cfg, "qk_layernorm", False), "Phi qk_layernorm variant unsupported"
    spec = DSModelSpec(arch="phi", vocab_size=cfg.vocab_size, hidden_size=H, num_layers=cfg.num_hidden_layers,
                       num_heads=nh, num_kv_heads=getattr(cfg, "num_key_value_heads", None) or nh,
                       intermediate_size=cfg.intermediate_size, norm="ln", norm_eps=cfg.layer_norm_eps, pos="rope",
                       rope_theta=theta, rotary_dim=int(hd * partial), act=cfg.hidden_act, gated_mlp=False,
                       qkv_bias=True, o_bias=True, mlp_bias=True, parallel_residual=True, shared_parallel_norm=True,
                       max_positions=cfg.max_position_embeddings, lm_head_bias=True,
                       tie_embeddings=bool(getattr(cfg, "tie_word_embeddings", False)))
    base = model.model
    layers = []
    for L in base.layers:
        a, mlp = L.self_attn, L.mlp
        layers.append(dict(ln1_w=L.input_layernorm.weight, ln1_b=L.input_layernorm.bias, q_w=a.q_proj.weight,
                           k_w=a.k_proj.weight, v_w=a.v_proj.weight, q_b=a.q_proj.bias, k_b=a.k_proj.bias,
                           v_b=a.v_proj.bias, o_w=a.dense.weight, o_b=a.dense.bias, fc1_w=mlp.fc1.weight,
                           fc1_b=mlp.fc1.bias, fc2_w=mlp.fc2.weight, fc2_b=mlp.fc2.bias))
    top = dict(embed=base.embed_tokens.weight, norm_w=base.final_layernorm.weight,
               norm_b=base.final_layernorm.bias, lm_head=model.lm_head.weight, lm_head_b=model.lm_head.bias)
    return spec, top, layers


def _megatron_parts(model):
    """(embedding, transformer stack) of a Megatron-LM GPT model, or None. Duck-typed on the attribute names the
    reference's policy keys on (`module_inject/containers/megatron_gpt.py:36-140`): Megatron is not a dependency."""
    lm = getattr(model, "language_model", None)
    if lm is None:
        return None
    emb = getattr(lm, "embedding", None)
    tr = getattr(lm, "encoder", None) or getattr(lm, "transformer", None)
    if emb is None or tr is None or not hasattr(emb, "word_embeddings") or not len(getattr(tr, "layers", [])):
        return None
    first = tr.layers[0]
    attn = getattr(first, "self_attention", None) or getattr(first, "attention", None)
    if attn is None or not hasattr(attn, "query_key_value") or not hasattr(first, "input_layernorm"):
        return None
    return emb, tr


def _megatron_gpt(model):
    """Megatron-LM GPT and GPT-MoE (reference containers `module_inject/containers/megatron_gpt.py`,
    `megatron_gpt_moe.py`; inference modules `ds_megatron_gpt.py`, `moe_inference.py`).

    * layers: `input_layernorm`, `self_attention.query_key_value` (`attention.` in the oldest Megatron sources) +
      `.dense`, `post_attention_layernorm`, `mlp.dense_h_to_4h` / `mlp.dense_4h_to_h`; learned positions, LayerNorm,
      tanh-GELU (Megatron's fused bias-gelu), LM head tied to the word embeddings.
    * fused QKV rows: Megatron v2 orders them [head, (q, k, v), head_dim]; older checkpoints [(q, k, v), head,
      head_dim] (`model.megatron_v2 = False`, reference `MegatronContainer.transpose_qkv_alignment`).
    * MoE layers (`mlp.deepspeed_moe`): top-1 gate `gate.wg`, experts `experts.deepspeed_experts[i]` as biased dense
      MLPs, output scaled by the gate probability; residual MoE (`mlp.moe.deepspeed_moe` + `mlp.mlp` +
      `mlp.coefficient`, PR-MoE) mixes the experts with a dense MLP. Every layer of the model must be of one kind
      (the inference stack is homogeneous); a dense / MoE mix raises.
    """
    emb, tr = _megatron_parts(model)
    first = tr.layers[0]
    old = not hasattr(first, "self_attention")
    attn0 = first.attention if old else first.self_attention
    V, H = emb.word_embeddings.weight.shape
    nh = getattr(attn0, "num_attention_heads", None) or attn0.num_attention_heads_per_partition
    hd = H // nh
    v2 = bool(getattr(model, "megatron_v2", not old))

    def experts_of(mlp):
        if hasattr(mlp, "deepspeed_moe"):
            return mlp.deepspeed_moe, None
        if hasattr(mlp, "moe") and hasattr(mlp.moe, "deepspeed_moe"):
            return mlp.moe.deepspeed_moe, mlp
        return None, None

    kinds = {("res" if experts_of(L.mlp)[1] is not None else "moe") if experts_of(L.mlp)[0] is not None else "dense"
             for L in tr.layers}
    if len(kinds) != 1:
        raise NotImplementedError(f"Megatron model mixes {sorted(kinds)} MLP layers: kernel injection needs every "
                                  f"layer to be of one kind")
    kind = kinds.pop()
    moe0, _ = experts_of(first.mlp)
    if moe0 is not None:
        ex0 = moe0.experts.deepspeed_experts
        E, I = len(ex0), ex0[0].dense_h_to_4h.weight.shape[0]
        k = int(getattr(moe0.gate, "k", 1))
    else:
        E, I, k = 0, first.mlp.dense_h_to_4h.weight.shape[0], 1
    spec = DSModelSpec(arch="megatron_gpt" + ("_moe" if E else ""), vocab_size=V, hidden_size=H,
                       num_layers=len(tr.layers), num_heads=nh, num_kv_heads=nh, intermediate_size=I, norm="ln",
                       norm_eps=float(getattr(first.input_layernorm, "eps", 1e-5)), pos="learned", act="gelu_tanh",
                       gated_mlp=False, qkv_bias=True, o_bias=True, mlp_bias=True,
                       max_positions=emb.position_embeddings.weight.shape[0], tie_embeddings=True, num_experts=E,
                       moe_top_k=k, moe_renormalize=False, moe_residual=kind == "res")
    layers = []
    for L in tr.layers:
        at = L.attention if old else L.self_attention
        w, b = at.query_key_value.weight, at.query_key_value.bias
        if v2:
            q, kk, v = _split_interleaved(w, nh, hd)
            qb, kb, vb = _split_interleaved(b, nh, hd)
        else:
            q, kk, v = w.split(H, 0)
            qb, kb, vb = b.split(H, 0)
        lw = dict(ln1_w=L.input_layernorm.weight, ln1_b=L.input_layernorm.bias,
                  ln2_w=L.post_attention_layernorm.weight, ln2_b=L.post_attention_layernorm.bias,
                  q_w=q, k_w=kk, v_w=v, q_b=qb, k_b=kb, v_b=vb, o_w=at.dense.weight, o_b=at.dense.bias)
        moe, outer = experts_of(L.mlp)
        if moe is None:
            lw.update(fc1_w=L.mlp.dense_h_to_4h.weight, fc1_b=L.mlp.dense_h_to_4h.bias,
                      fc2_w=L.mlp.dense_4h_to_h.weight, fc2_b=L.mlp.dense_4h_to_h.bias)
        else:
            ex = moe.experts.deepspeed_experts
            lw.update(router_w=moe.gate.wg.weight,
                      experts_fc1=torch.stack([e.dense_h_to_4h.weight for e in ex]),
                      experts_fc1_b=torch.stack([e.dense_h_to_4h.bias for e in ex]),
                      experts_down=torch.stack([e.dense_4h_to_h.weight for e in ex]),
                      experts_down_b=torch.stack([e.dense_4h_to_h.bias for e in ex]))
            if outer is not None:
                lw.update(res_fc1_w=outer.mlp.dense_h_to_4h.weight, res_fc1_b=outer.mlp.dense_h_to_4h.bias,
                          res_fc2_w=outer.mlp.dense_4h_to_h.weight, res_fc2_b=outer.mlp.dense_4h_to_h.bias,
                          coef_w=outer.coefficient.weight, coef_b=getattr(outer.coefficient, "bias", None))
        layers.append(lw)
    fl = tr.final_layernorm
    top = dict(embed=emb.word_embeddings.weight, pos_embed=emb.position_embeddings.weight, norm_w=fl.weight,
               norm_b=fl.bias, lm_head=emb.word_embeddings.weight)
    return spec, top, layers


CONVERTERS = {
    "llama": _llama_like, "mistral": _llama_like, "qwen2": _llama_like, "internlm": _llama_like,
    "gpt2": _gpt2, "bloom": _bloom, "opt": _opt, "gpt_neox": _gpt_neox, "gptj": _gptj,
    "mixtral": _mixtral, "falcon": _falcon, "phi": _phi, "gpt_neo": _gpt_neo,
}


def supported(model):
    from ...models.llama import LlamaForCausalLM as NativeLlama
    if isinstance(model, NativeLlama):
        return True
    if _megatron_parts(model) is not None:
        return True
    mt = getattr(getattr(model, "config", None), "model_type", None)
    return mt in CONVERTERS


def extract(model):
    from ...models.llama import LlamaForCausalLM as NativeLlama
    if isinstance(model, NativeLlama):
        return _native_llama(model)
    if _megatron_parts(model) is not None:
        return _megatron_gpt(model)
    mt = model.config.model_type
    if mt not in CONVERTERS:
        raise NotImplementedError(f"no kernel-injection policy for model_type={mt!r}")
    return CONVERTERS[mt](model)


# ------------------------------------------------------------------------------------------------ TP sharding
def _rows(w, r, tp):
    n = w.shape[0] // tp
    return w[r * n:(r + 1) * n]


def _cols(w, r, tp):
    n = w.shape[1] // tp
    return w[:, r * n:(r + 1) * n]


def _kv_rows(w, spec, r, tp):
    """k/v rows for rank r: a contiguous slice of kv heads, or the single kv head its q heads map to."""
    if w is None:
        return None
    D = spec.head_dim
    if spec.num_kv_heads >= tp:
        return _rows(w, r, tp)
    group = spec.num_heads // spec.num_kv_heads
    kv = (r * (spec.num_heads // tp)) // group
    return w[kv * D:(kv + 1) * D]


def shard_layer(spec, lw, r, tp):
    out = {}
    q = _rows(lw["q_w"], r, tp)
    k = _kv_rows(lw["k_w"], spec, r, tp)
    v = _kv_rows(lw["v_w"], spec, r, tp)
    out["qkv_w"] = torch.cat([q, k, v], 0)
    if lw.get("q_b") is not None:
        out["qkv_b"] = torch.cat([_rows(lw["q_b"], r, tp), _kv_rows(lw["k_b"], spec, r, tp),
                                  _kv_rows(lw["v_b"], spec, r, tp)], 0)
    out["o_w"] = _cols(lw["o_w"], r, tp)
    if lw.get("o_b") is not None:
        out["o_b"] = lw["o_b"]
    if "experts_gate_up" in lw:  # [E, 2I, H] gate rows then up rows; [E, H, I]
        gu = lw["experts_gate_up"]
        I = gu.shape[1] // 2
        n = I // tp
        out["fc1_w"] = torch.cat([gu[:, r * n:(r + 1) * n], gu[:, I + r * n:I + (r + 1) * n]], 1)
        out["fc2_w"] = lw["experts_down"][:, :, r * n:(r + 1) * n]
        out["router_w"] = lw["router_w"]
    elif "experts_fc1" in lw:  # Megatron-style experts: plain biased MLPs [E, I, H] / [E, H, I]
        n = lw["experts_fc1"].shape[1] // tp
        out["fc1_w"] = lw["experts_fc1"][:, r * n:(r + 1) * n]
        out["fc1_b"] = lw["experts_fc1_b"][:, r * n:(r + 1) * n]
        out["fc2_w"] = lw["experts_down"][:, :, r * n:(r + 1) * n]
        out["fc2_b"] = lw["experts_down_b"] / tp  # every TP rank adds its share; the all-reduce restores the bias
        out["router_w"] = lw["router_w"]
        if "res_fc1_w" in lw:
            out["res_fc1_w"], out["res_fc1_b"] = _rows(lw["res_fc1_w"], r, tp), _rows(lw["res_fc1_b"], r, tp)
            out["res_fc2_w"], out["res_fc2_b"] = _cols(lw["res_fc2_w"], r, tp), lw["res_fc2_b"]
            out["coef_w"] = lw["coef_w"]
            if lw.get("coef_b") is not None:
                out["coef_b"] = lw["coef_b"]
    elif "gate_w" in lw:
        out["fc1_w"] = torch.cat([_rows(lw["gate_w"], r, tp), _rows(lw["up_w"], r, tp)], 0)
        if lw.get("gate_b") is not None:
            out["fc1_b"] = torch.cat([_rows(lw["gate_b"], r, tp), _rows(lw["up_b"], r, tp)], 0)
    else:
        out["fc1_w"] = _rows(lw["fc1_w"], r, tp)
        if lw.get("fc1_b") is not None:
            out["fc1_b"] = _rows(lw["fc1_b"], r, tp)
    if "experts_down" not in lw:
        out["fc2_w"] = _cols(lw["fc2_w"], r, tp)
    if lw.get("fc2_b") is not None and "experts_down" not in lw:
        out["fc2_b"] = lw["fc2_b"]
    for n in ("ln1_w", "ln1_b", "ln2_w", "ln2_b"):
        if lw.get(n) is not None:
            out[n] = lw[n]
    if spec.shared_parallel_norm:
        out["ln2_w"], out["ln2_b"] = lw["ln1_w"], lw.get("ln1_b")
    return out


def _put(param, src):
    if param is None or src is None:
        return
    param.data.copy_(src.detach().to(param.dtype))


def load_layer(model: DSInferenceModel, idx, lw):
    """Canonical full weights of layer `idx` -> this rank's shard of the injected layer."""
    for name, t in shard_layer(model.spec, lw, model.tp_rank, model.tp_size).items():
        _put(getattr(model.layers[idx], name), t)


def load_top(model: DSInferenceModel, top):
    """Embeddings, final norm and LM head (vocab rows sharded over the ranks, zero-padded)."""
    spec, r = model.spec, model.tp_rank
    _put(model.embed, top["embed"])
    if model.pos_embed is not None:
        pe = top["pos_embed"]
        model.pos_embed.data.zero_()
        n = min(pe.shape[0], model.pos_embed.shape[0])
        model.pos_embed.data[:n].copy_(pe[:n].to(model.dtype))
    if spec.embed_norm:
        _put(model.embed_ln_w, top["embed_ln_w"])
        _put(model.embed_ln_b, top["embed_ln_b"])
    _put(model.norm_w, top["norm_w"])
    _put(model.norm_b, top.get("norm_b"))
    V, vl = spec.vocab_size, model.vocab_local
    lm = top["lm_head"]
    model.lm_head.data.zero_()
    lo, hi = r * vl, min((r + 1) * vl, V)
    if hi > lo:
        model.lm_head.data[:hi - lo].copy_(lm[lo:hi].to(model.dtype))
        if model.lm_head_b is not None and top.get("lm_head_b") is not None:
            model.lm_head_b.data.zero_()
            model.lm_head_b.data[:hi - lo].copy_(top["lm_head_b"][lo:hi].to(model.dtype))


def load_into(model: DSInferenceModel, top, layers):
    for i, lw in enumerate(layers[:len(model.layers)]):
        load_layer(model, i, lw)
    load_top(model, top)


def spec_from_config(hf_config):
    """The `DSModelSpec` of a HF config alone: the architecture is instantiated on the meta device (no weight
    memory) and read by its converter."""
    import transformers
    with torch.device("meta"):
        skeleton = transformers.AutoModelForCausalLM.from_config(hf_config)
    return extract(skeleton)[0]


def from_model(model, tp_group=None, tp_size=1, tp_rank=0, dtype=torch.bfloat16, device=None, max_positions=None):
    spec, top, layers = extract(model)
    if max_positions:
        spec.max_positions = max(spec.max_positions, max_positions)
    ds = DSInferenceModel(spec, tp_group, tp_size, tp_rank, dtype, device)
    with torch.no_grad():
        load_into(ds, top, layers)
    return ds
