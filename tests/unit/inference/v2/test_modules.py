"""Inference v2 building blocks (`inference/v2/modules`): a two-layer Llama-style decoder assembled ONLY from the
module interfaces (heuristics -> registered implementations) runs a prompt step and a decode step over a ragged batch
and matches a dense fp32 PyTorch model of the same weights; registry / config validation."""
import math

import pytest
import torch
import torch.nn.functional as F

from deepspeedsyclsupport_amd.inference.v2.inference_utils import ActivationType, DtypeEnum, NormTypeEnum
from deepspeedsyclsupport_amd.inference.v2.modules import (ConfigBundle, DSEmbeddingsConfig, DSLinearConfig,
                                                           DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                                                           DSUnembedConfig, PositionalEmbeddingType, RotateHalfConfig,
                                                           heuristics)
from deepspeedsyclsupport_amd.inference.v2.modules.interfaces import DSLinearBase, DSLinearRegistry
from deepspeedsyclsupport_amd.inference.v2.ragged import DSSequenceDescriptor, RaggedBatchWrapper

CASES = [pytest.param("cpu", torch.float32, id="cpu-fp32"),
         pytest.param("cuda", torch.bfloat16, id="gpu-bf16", marks=pytest.mark.gpu)]
V, H, HQ, HK, D, I, L, BS = 96, 256, 4, 2, 64, 512, 2, 16


def _weights(dtype, device):
    g = torch.Generator().manual_seed(0)

    def r(*s, scale=0.05):
        return (torch.randn(*s, generator=g) * scale).to(dtype).to(device)

    w = {"emb": r(V, H, scale=0.5), "norm": (1 + r(H)), "layers": []}
    for _ in range(L):
        w["layers"].append({"ln1": 1 + r(H), "qkv": r((HQ + 2 * HK) * D, H), "o": r(H, HQ * D), "ln2": 1 + r(H),
                            "gate_up": r(2 * I, H), "down": r(H, I)})
    return w


def _dense_reference(w, ids):
    """fp32 causal decoder over one full sequence ids [n] -> logits of the last token."""
    f = lambda t: t.float().cpu()
    x = f(w["emb"])[ids]
    n = ids.numel()
    inv = 1.0 / (10000.0**(torch.arange(0, D, 2, dtype=torch.float64) / D))
    ang = torch.outer(torch.arange(n, dtype=torch.float64), inv)
    cos, sin = ang.cos().float()[:, None], ang.sin().float()[:, None]

    def rope(t):
        a, b = t[..., :D // 2], t[..., D // 2:]
        return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

    def rms(t, g):
        return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + 1e-5) * f(g)

    for lw in w["layers"]:
        h = rms(x, lw["ln1"])
        q, k, v = (h @ f(lw["qkv"]).t()).view(n, HQ + 2 * HK, D).split([HQ, HK, HK], 1)
        q, k = rope(q), rope(k)
        k, v = k.repeat_interleave(HQ // HK, 1), v.repeat_interleave(HQ // HK, 1)
        sc = torch.einsum("nhd,mhd->hnm", q, k) / math.sqrt(D)
        sc = sc.masked_fill(torch.ones(n, n).triu(1).bool()[None], float("-inf"))
        a = torch.einsum("hnm,mhd->nhd", sc.softmax(-1), v).reshape(n, HQ * D)
        x = x + a @ f(lw["o"]).t()
        h = rms(x, lw["ln2"])
        gu = h @ f(lw["gate_up"]).t()
        x = x + (F.silu(gu[:, :I]) * gu[:, I:]) @ f(lw["down"]).t()
    return rms(x[-1:], w["norm"]) @ f(w["emb"]).t()


@pytest.mark.parametrize("device,dtype", CASES)
def test_decoder_from_modules(device, dtype):
    de = DtypeEnum(dtype)
    w = _weights(dtype, device)
    mt = 256
    embed = heuristics.instantiate_embed(DSEmbeddingsConfig(max_tokens=mt, residual_dtype=de, embedding_dim=H))
    norm = heuristics.instantiate_pre_norm(DSNormConfig(max_tokens=mt, type=NormTypeEnum.RMSNorm, channels=H,
                                                        residual_dtype=de, input_dtype=de, output_dtype=de))
    assert type(norm).name() == "cuda_pre_rms"
    attn = heuristics.instantiate_attention(DSSelfAttentionConfig(
        max_tokens=mt, n_heads_q=HQ, n_heads_kv=HK, head_size=D, max_sequences=8, scale_factor=1 / math.sqrt(D),
        input_dtype=de, output_dtype=de, positional_embedding_type=PositionalEmbeddingType.rotate_half,
        positional_embedding_config=RotateHalfConfig(theta_base=10000.0)))
    lin = lambda i, o, act=ActivationType.IDENTITY: heuristics.instantiate_linear(DSLinearConfig(
        max_tokens=mt, in_channels=i, out_channels=o, activation=act, input_dtype=de, output_dtype=de))
    qkv_l, o_l = lin(H, (HQ + 2 * HK) * D), lin(HQ * D, H)
    up_l, down_l = lin(H, I, ActivationType.SiGLU), lin(I, H)
    unembed = heuristics.instantiate_unembed(DSUnembedConfig(max_tokens=mt, dtype=de, norm_type=NormTypeEnum.RMSNorm,
                                                             model_dim=H, max_sequences=8, vocab_size=V))
    caches = [(torch.zeros(16, HK, BS, D, device=device, dtype=dtype),
               torch.zeros(16, HK, BS, D, device=device, dtype=dtype)) for _ in range(L)]
    batch = RaggedBatchWrapper(block_size=BS, device=torch.device(device))
    seqs = {1: DSSequenceDescriptor(1, BS), 2: DSSequenceDescriptor(2, BS)}
    free = [0]
    g = torch.Generator().manual_seed(5)
    full = {1: torch.randint(0, V, (19, ), generator=g), 2: torch.randint(0, V, (7, ), generator=g)}

    def put(items):
        batch.clear()
        for u, toks in items:
            s = seqs[u]
            need = s.blocks_needed(toks.numel())
            s.extend_kv_cache(range(free[0], free[0] + need))
            free[0] += need
            s.pre_forward(toks.numel())
            batch.insert_sequence(s, toks)
        batch.finalize()
        resid = embed(batch, w["emb"])
        hidden = None
        for lw, kv in zip(w["layers"], caches):
            resid, hidden = norm(resid, hidden, lw["ln1"])
            hidden = o_l(attn(qkv_l(hidden, lw["qkv"]), kv, batch), lw["o"])
            resid, hidden = norm(resid, hidden, lw["ln2"])
            hidden = down_l(up_l(hidden, lw["gate_up"]), lw["down"])
        resid = resid + hidden
        logits = batch.restore_order(unembed(resid, w["emb"], batch, gamma=w["norm"]))
        for u, _ in items:
            seqs[u].post_forward()
        return logits.float().cpu()

    tol = dict(rtol=5e-2, atol=8e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    out = put([(1, full[1][:18]), (2, full[2])])
    torch.testing.assert_close(out[0:1], _dense_reference(w, full[1][:18]), **tol)
    torch.testing.assert_close(out[1:2], _dense_reference(w, full[2]), **tol)
    out = put([(1, full[1][18:])])                    # one decode step on the cached prefix
    torch.testing.assert_close(out, _dense_reference(w, full[1]), **tol)


@pytest.mark.parametrize("device,dtype", CASES)
def test_moe_module(device, dtype):
    from deepspeedsyclsupport_amd.ops import moe_ops
    de = DtypeEnum(dtype)
    E, k, Hm, Im = 4, 2, 128, 256
    moe = heuristics.instantiate_moe(DSMoEConfig(max_tokens=64, model_dim=Hm, intermediate_features=Im, n_experts=E,
                                                 top_k=k, input_dtype=de, output_dtype=de,
                                                 activation=ActivationType.SiGLU, normalize_scores=True))
    torch.manual_seed(3)
    x = torch.randn(24, Hm, device=device, dtype=dtype)
    gate = torch.randn(E, Hm, device=device, dtype=dtype)
    w1 = torch.randn(E, 2 * Im, Hm, device=device, dtype=dtype) * 0.05
    w2 = torch.randn(E, Hm, Im, device=device, dtype=dtype) * 0.05
    out = moe(x, moe.transform_gate_param(gate), w1, w2)
    act = lambda h: F.silu(h[..., :Im]) * h[..., Im:]
    ref = moe_ops.moe_block_reference(x.float(), gate.float(), w1.float(), w2.float(), k, act, True)
    torch.testing.assert_close(out.float(), ref, **(dict(rtol=5e-2, atol=5e-2) if dtype == torch.bfloat16 else
                                                    dict(rtol=1e-4, atol=1e-4)))


def test_registry_rules():
    cfg = DSLinearConfig(max_tokens=8, in_channels=16, out_channels=16, input_dtype="bf16", output_dtype="fp16")
    assert cfg.input_dtype is DtypeEnum.bf16
    with pytest.raises(ValueError, match="not supported"):      # mixed in / out dtypes
        DSLinearRegistry.instantiate_config(ConfigBundle(name="blas_fp_linear", config=cfg))
    with pytest.raises(KeyError):
        DSLinearRegistry.instantiate_config(ConfigBundle(name="no_such_linear", config=cfg))
    with pytest.raises(TypeError):
        DSLinearRegistry.register_module(torch.nn.Linear)

    @DSLinearRegistry.register_module
    class Doubling(DSLinearBase):

        @staticmethod
        def name():
            return "doubling_linear"

        @staticmethod
        def supports_config(config):
            return True

        def forward(self, hidden_states, w, b=None):
            return 2 * F.linear(hidden_states, w, b)

    m = DSLinearRegistry.instantiate_config(ConfigBundle(name="doubling_linear", config=cfg))
    x, wt = torch.randn(3, 16), torch.randn(16, 16)
    torch.testing.assert_close(m(x, wt), 2 * x @ wt.t())
    del DSLinearRegistry.registry["doubling_linear"]
