"""Encoder kernel injection (reference `tests/unit/inference/test_inference.py` bert / distilbert / roberta
fill-mask and classification cases): `init_inference(..., replace_with_kernel_inject=True)` swaps the encoder layers
for fused `DSEncoderLayer`s and the task output must match the HF model — with padding masks, under TP=2 (gloo)
and on the GPU in bf16. HF models are tiny random-init instances (no checkpoints)."""
import copy

import pytest
import torch

from ..common import run_distributed

transformers = pytest.importorskip("transformers")
V = 300


def tiny(kind, H=64, heads=4):
    T = transformers
    torch.manual_seed(0)
    if kind == "bert":
        c = T.BertConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2, num_attention_heads=heads,
                         intermediate_size=4 * H, max_position_embeddings=64)
        return T.BertForMaskedLM(c)
    if kind == "bert_cls":
        c = T.BertConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2, num_attention_heads=heads,
                         intermediate_size=4 * H, max_position_embeddings=64, num_labels=3)
        return T.BertForSequenceClassification(c)
    if kind == "roberta":
        c = T.RobertaConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2, num_attention_heads=heads,
                            intermediate_size=4 * H, max_position_embeddings=70, pad_token_id=1)
        return T.RobertaForMaskedLM(c)
    if kind == "distilbert":
        c = T.DistilBertConfig(vocab_size=V, dim=H, n_layers=2, n_heads=heads, hidden_dim=4 * H,
                               max_position_embeddings=64)
        return T.DistilBertForMaskedLM(c)
    if kind == "clip_text":
        c = T.CLIPTextConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2, num_attention_heads=heads,
                             intermediate_size=4 * H, max_position_embeddings=64, eos_token_id=2)
        return T.CLIPTextModel(c)
    if kind == "clip_vision":
        c = T.CLIPVisionConfig(hidden_size=H, num_hidden_layers=2, num_attention_heads=heads, intermediate_size=4 * H,
                               image_size=32, patch_size=8)
        return T.CLIPVisionModel(c)
    raise ValueError(kind)


def _inputs(B=3, S=17):
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, V, (B, S), generator=g)
    mask = torch.ones(B, S, dtype=torch.long)
    mask[1, 11:] = 0
    mask[2, 5:] = 0
    return ids, mask


def _out(o):
    return o.logits if hasattr(o, "logits") else o[0]


@pytest.mark.parametrize("kind", ["clip_text", "clip_vision"])
def test_clip_inject_parity_cpu(kind):
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind).eval()
    if kind == "clip_text":
        ids, mask = _inputs()
        kw = dict(input_ids=ids, attention_mask=mask)
    else:
        kw = dict(pixel_values=torch.randn(2, 3, 32, 32, generator=torch.Generator().manual_seed(3)))
    with torch.no_grad():
        ref = m(**kw)
    eng = ds.init_inference(copy.deepcopy(m), dtype=torch.float32, replace_with_kernel_inject=True)
    assert eng.encoder_injected == 2
    with torch.no_grad():
        out = eng(**kw)
    a, b = out.last_hidden_state, ref.last_hidden_state
    if kind == "clip_text":
        valid = kw["attention_mask"].bool()
        a, b = a[valid], b[valid]
    assert (a - b).abs().max().item() < 1e-4
    assert (out.pooler_output - ref.pooler_output).abs().max().item() < 1e-4


@pytest.mark.parametrize("kind", ["bert", "bert_cls", "roberta", "distilbert"])
def test_encoder_inject_parity_cpu(kind):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.module_inject.encoder import DSEncoderLayer
    m = tiny(kind).eval()
    ids, mask = _inputs()
    with torch.no_grad():
        ref = _out(m(input_ids=ids, attention_mask=mask))
    eng = ds.init_inference(copy.deepcopy(m), dtype=torch.float32, replace_with_kernel_inject=True)
    assert eng.encoder_injected == 2
    assert sum(isinstance(x, DSEncoderLayer) for x in eng.module.modules()) == 2
    with torch.no_grad():
        out = _out(eng(input_ids=ids, attention_mask=mask))
    valid = mask.bool() if out.dim() == 3 else slice(None)
    err = (out[valid] - ref[valid]).abs().max().item()
    assert err < 1e-4, f"{kind}: {err}"


def _tp_run(kind):
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind).eval()
    ids, mask = _inputs()
    with torch.no_grad():
        ref = _out(m(input_ids=ids, attention_mask=mask))
    eng = ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=True, tensor_parallel={"tp_size": 2})
    assert eng.encoder_injected == 2
    with torch.no_grad():
        out = _out(eng(input_ids=ids, attention_mask=mask))
    valid = mask.bool() if out.dim() == 3 else slice(None)
    err = (out[valid] - ref[valid]).abs().max().item()
    assert err < 1e-4, f"{kind} tp2: {err}"


@pytest.mark.parametrize("kind", ["bert", "distilbert"])
def test_encoder_inject_tp2(kind):
    run_distributed(_tp_run, 2, kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bert", "roberta", "distilbert", "clip_text"])
def test_encoder_inject_bf16_gpu(kind):
    import deepspeedsyclsupport_amd as ds
    m = tiny(kind, H=256, heads=4).eval()
    ids, mask = _inputs(B=4, S=64)
    with torch.no_grad():
        ref = _out(m(input_ids=ids, attention_mask=mask)).float()
    eng = ds.init_inference(copy.deepcopy(m), dtype=torch.bfloat16, replace_with_kernel_inject=True)
    from deepspeedsyclsupport_amd.ops import flash_small as FS
    calls = []
    orig = FS.FlashSmallFunc.apply

    def spy(*a):
        calls.append((a[3] is not None, a[4] is not None))
        return orig(*a)

    FS.FlashSmallFunc.apply = spy
    try:
        with torch.no_grad():
            out = _out(eng(input_ids=ids.cuda(), attention_mask=mask.cuda())).float().cpu()
    finally:
        FS.FlashSmallFunc.apply = orig
    valid = mask.bool()
    assert (out[valid] - ref[valid]).abs().max().item() < 0.05 * ref.abs().max().item() + 0.05
    # head dim 64: both layers' attention ran on the in-tree kernel with the padding mask as a bias, not on SDPA
    assert len(calls) == 2 and all(b1 or b2 for b1, b2 in calls), calls
    if kind != "clip_text":
        assert all(b1 and not b2 for b1, b2 in calls), calls  # a pure padding mask is the per-key bias
