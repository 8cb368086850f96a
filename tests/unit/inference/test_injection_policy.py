"""User-specified tensor parallelism: `init_inference(model, injection_policy={Block: ("attn.out", "mlp.fc2")})`
(reference `inference/engine.py:135-154`, `module_inject/replace_module.py:266-300`), the structural policy parser
(`auto_tp.py:271-311`) and the shard-size / fused-QKV helpers (`tp_shard.py`, `fusedqkv_utils.py`)."""
import pytest
import torch
import torch.nn as nn

from ..common import run_distributed


class _Block(nn.Module):

    def __init__(self, H=32, heads=4):
        super().__init__()
        self.ln1 = nn.LayerNorm(H)
        self.q, self.k, self.v = nn.Linear(H, H), nn.Linear(H, H), nn.Linear(H, H)
        self.merge = nn.Linear(H, H)       # deliberately not a name the heuristics know
        self.ln2 = nn.LayerNorm(H)
        self.up = nn.Linear(H, 4 * H)
        self.shrink = nn.Linear(4 * H, H)
        self.num_heads = heads

    def forward(self, x):
        h = self.ln1(x)
        B, S, H = h.shape
        hd = self.q.out_features // self.num_heads

        def heads(t):
            return t.view(B, S, self.num_heads, -1).transpose(1, 2)

        a = torch.nn.functional.scaled_dot_product_attention(heads(self.q(h)), heads(self.k(h)), heads(self.v(h)))
        del hd
        x = x + self.merge(a.transpose(1, 2).reshape(B, S, -1))
        return x + self.shrink(torch.nn.functional.gelu(self.up(self.ln2(x))))


class _Net(nn.Module):

    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(50, 32)
        self.layers = nn.ModuleList([_Block() for _ in range(2)])
        self.head = nn.Linear(32, 50)

    def forward(self, ids):
        x = self.emb(ids)
        for blk in self.layers:
            x = blk(x)
        return self.head(x)


def _policy_run(use_parser):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.module_inject.auto_tp import AutoTP
    from deepspeedsyclsupport_amd.module_inject.layers import LinearAllreduce, LinearLayer
    torch.manual_seed(0)
    m = _Net().eval()
    ids = torch.randint(0, 50, (2, 9))
    with torch.no_grad():
        ref = m(ids)
    if use_parser:
        policy = dict(AutoTP.tp_parser(m))
        assert set(policy[_Block]) == {"merge", "shrink"}, policy   # the last linear before each norm / block end
    else:
        policy = {_Block: ("merge", "shrink")}
    eng = ds.init_inference(m, dtype=torch.float32, tensor_parallel={"tp_size": 2}, injection_policy=policy)
    blk = eng.module.layers[0]
    assert isinstance(blk.merge, LinearAllreduce) and isinstance(blk.shrink, LinearAllreduce)
    assert isinstance(blk.q, LinearLayer) and blk.q.weight.shape == (16, 32) and blk.num_heads == 2
    assert isinstance(eng.module.head, nn.Linear)      # outside the listed blocks: untouched
    with torch.no_grad():
        out = eng(ids)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("use_parser", [False, True])
def test_user_injection_policy_tp2(use_parser):
    run_distributed(_policy_run, 2, use_parser)


def test_injection_policy_validation():
    from deepspeedsyclsupport_amd.module_inject.auto_tp import AutoTP
    m = _Net()
    with pytest.raises(ValueError, match="not valid"):
        AutoTP(m, None, 2, 0, injection_policy={_Block: ("no_such_linear", )}).apply()
    with pytest.raises(TypeError):
        AutoTP(m, None, 2, 0, injection_policy={"Block": ("merge", )})
    import deepspeedsyclsupport_amd as ds
    with pytest.raises(ValueError, match="both"):
        ds.init_inference(m, dtype=torch.float32, replace_with_kernel_inject=True,
                          injection_policy={_Block: ("merge", )})


def test_shard_sizes_and_fused_qkv():
    from deepspeedsyclsupport_amd.module_inject import tp_shard
    from deepspeedsyclsupport_amd.module_inject.fusedqkv_utils import (prepare_tp_fused_qkvw, require_tp_fused_qkvw,
                                                                     split_by_qkvlist_and_refuse)
    tp_shard.set_num_kv_heads(None)
    assert tp_shard.get_shard_size_list(12, 4) == [3, 3, 3, 3]
    with pytest.raises(AssertionError):
        tp_shard.get_shard_size(10, 4, 0)
    tp_shard.set_num_kv_heads(6)       # 6 kv heads over 4 ranks: 2, 2, 1, 1 heads
    assert tp_shard.get_shard_size_list(6 * 8, 4) == [16, 16, 8, 8]
    tp_shard.set_num_kv_heads(None)
    assert require_tp_fused_qkvw("h.0.attn.c_attn.weight", 2) and not require_tp_fused_qkvw("h.0.attn.c_proj", 2)
    H = 8
    q, k, v = [torch.full((H, 2), float(i)) + torch.arange(H)[:, None] / 100 for i in range(3)]
    fused = torch.cat([q, k, v])
    s1 = prepare_tp_fused_qkvw("c_attn", fused, 2, 1)
    torch.testing.assert_close(s1, torch.cat([q[4:], k[4:], v[4:]]))
    inter = torch.stack([q.view(4, 2, 2), k.view(4, 2, 2), v.view(4, 2, 2)], 1).reshape(3 * H, 2)  # [head, qkv, D]
    s0 = prepare_tp_fused_qkvw("query_key_value", inter, 2, 0)
    torch.testing.assert_close(s0, inter[:12])
    parts = split_by_qkvlist_and_refuse([q, k, v], 4)
    torch.testing.assert_close(parts[1], torch.cat([q[4:], k[4:], v[4:]]))


def test_bloom_alibi_matches_transformers():
    from transformers.models.bloom.modeling_bloom import build_alibi_tensor

    from deepspeedsyclsupport_amd.module_inject.auto_tp_model_utils import build_bloom_alibi_tensor
    mask = torch.ones(2, 7, dtype=torch.long)
    mask[1, :2] = 0
    for heads in (8, 12):
        torch.testing.assert_close(build_bloom_alibi_tensor(mask, heads, torch.float32),
                                   build_alibi_tensor(mask, heads, torch.float32))


def _bloom_tp(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from .test_inference import tiny
    dist.init_distributed("gloo")
    m = tiny("bloom").eval()
    ids = torch.randint(0, m.config.vocab_size, (2, 9), generator=torch.Generator().manual_seed(1))
    mask = torch.ones_like(ids)
    mask[1, :3] = 0                                    # left padding: ALiBi positions follow the mask
    with torch.no_grad():
        ref = m(ids, attention_mask=mask, use_cache=False).logits
    eng = ds.init_inference(m, dtype=torch.float32, tensor_parallel={"tp_size": 2})
    assert "build_alibi_tensor" in vars(eng.module.transformer)      # the per-rank builder is in place
    with torch.no_grad():
        got = eng.module(ids, attention_mask=mask, use_cache=False).logits
    if dist.get_rank() == 0:
        torch.save({"ref": ref, "got": got}, out)


def test_auto_tp_bloom_alibi_per_rank(tmp_path):
    """HF BLOOM under AutoTP (no kernel injection), 2 ranks: each rank's attention gets the ALiBi rows of its own
    heads, and the logits equal the unsharded model's."""
    from ..common import run_distributed
    out = str(tmp_path / "r.pt")
    run_distributed(_bloom_tp, 2, out)
    r = torch.load(out, weights_only=True)
    torch.testing.assert_close(r["got"][0], r["ref"][0], rtol=2e-4, atol=2e-4)
    torch.testing.assert_close(r["got"][1, 3:], r["ref"][1, 3:], rtol=2e-4, atol=2e-4)
