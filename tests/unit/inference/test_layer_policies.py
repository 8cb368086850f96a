"""Per-layer kernel injection through policies (`module_inject/policy.py`, `module_inject/containers.py`; reference
`module_inject/containers/*.py`, `replace_module.py:182-360`): `init_inference(model, injection_policy={Layer:
Policy})` swaps each client layer for one fused inference layer built from what the policy reads; a user-defined
policy does the same for an architecture the framework has never seen."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from .test_inference import tiny


def _layer_cls(kind):
    import transformers.models as M
    return {"llama": M.llama.modeling_llama.LlamaDecoderLayer, "gpt2": M.gpt2.modeling_gpt2.GPT2Block,
            "opt": M.opt.modeling_opt.OPTDecoderLayer, "gpt_neox": M.gpt_neox.modeling_gpt_neox.GPTNeoXLayer,
            "bloom": M.bloom.modeling_bloom.BloomBlock, "gptj": M.gptj.modeling_gptj.GPTJBlock,
            "gpt_neo": M.gpt_neo.modeling_gpt_neo.GPTNeoBlock}[kind]


@pytest.mark.parametrize("kind,policy", [("llama", "LLAMALayerPolicy"), ("gpt2", "HFGPT2LayerPolicy"),
                                         ("opt", "HFOPTLayerPolicy"), ("gpt_neox", "GPTNEOXLayerPolicy"),
                                         ("bloom", "BLOOMLayerPolicy"), ("gptj", "HFGPTJLayerPolicy"),
                                         ("gpt_neo", "HFGPTNEOLayerPolicy")])
def test_hf_layers_replaced_through_policies(kind, policy):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.module_inject import containers as C
    m = tiny(kind).eval()
    ids = torch.randint(0, m.config.vocab_size, (2, 12), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = m(ids, use_cache=False).logits
    eng = ds.init_inference(m, dtype=torch.float32, injection_policy={_layer_cls(kind): getattr(C, policy)})
    n_layers = getattr(m.config, "num_hidden_layers", None) or m.config.num_layers
    assert eng.policy_injected == n_layers
    assert not any(isinstance(x, _layer_cls(kind)) for x in eng.module.modules())
    with torch.no_grad():
        out = eng(ids, use_cache=False).logits
    torch.testing.assert_close(out, ref, rtol=2e-4, atol=2e-4)


class _Block(nn.Module):
    """A pre-norm decoder block with its own naming and a ReLU MLP."""

    def __init__(self, H=64, heads=4):
        super().__init__()
        self.n1, self.n2 = nn.LayerNorm(H), nn.LayerNorm(H)
        self.wqkv, self.wo = nn.Linear(H, 3 * H), nn.Linear(H, H)
        self.a, self.b = nn.Linear(H, 2 * H), nn.Linear(2 * H, H)
        self.heads = heads

    def forward(self, x):
        B, S, H = x.shape
        q, k, v = self.wqkv(self.n1(x)).view(B, S, 3, self.heads, -1).permute(2, 0, 3, 1, 4)
        x = x + self.wo(F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, S, H))
        return x + self.b(F.relu(self.a(self.n2(x))))


def test_user_defined_policy():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.module_inject.policy import TransformerPolicy
    from deepspeedsyclsupport_amd.utils.types import ActivationFuncType

    class MyPolicy(TransformerPolicy):

        def __init__(self, client_module, inference=True):
            super().__init__(inference, mlp_act_func_type=ActivationFuncType.ReLU)
            self.client_module = client_module

        def get_hidden_heads(self):
            c = self.client_module
            return c.wo.in_features, c.heads, c.n1.eps, c.a.out_features

        def attention(self, enable_training=False):
            c = self.client_module
            return c.wqkv.weight, c.wqkv.bias, c.wo.weight, c.wo.bias

        def mlp(self, enable_training=False):
            c = self.client_module
            return c.a.weight, c.a.bias, c.b.weight, c.b.bias

        def layernorm(self):
            c = self.client_module
            return c.n2.weight, c.n2.bias, c.n1.weight, c.n1.bias

    torch.manual_seed(0)
    net = nn.Sequential(_Block(), _Block()).eval()
    x = torch.randn(2, 9, 64)
    with torch.no_grad():
        ref = net(x)
    eng = ds.init_inference(net, dtype=torch.float32, injection_policy={_Block: MyPolicy})
    assert eng.policy_injected == 2
    with torch.no_grad():
        torch.testing.assert_close(eng(x), ref, rtol=1e-4, atol=1e-4)


def test_policy_tables_and_readers():
    from deepspeedsyclsupport_amd.module_inject import containers as C
    from deepspeedsyclsupport_amd.module_inject.replace_policy import generic_policies, replace_policies
    from deepspeedsyclsupport_amd.module_inject.utils import policy_to_ds_container
    assert C.LLAMALayerPolicy in replace_policies and C.UNetPolicy in generic_policies
    m = tiny("llama")
    layer = m.model.layers[0]
    pol = C.LLAMALayerPolicy(layer)
    H = m.config.hidden_size
    qkvw, qkvb, ow, ob = pol.attention()
    assert qkvw.shape == (H + 2 * (H // 2), H) and qkvb is None and ow.shape == (H, H) and pol.num_kv == 2
    iw, _, o2, _ = pol.mlp()
    torch.testing.assert_close(iw[:2 * H], layer.mlp.gate_proj.weight)
    cont = policy_to_ds_container(policy=pol, config=None, model_config=m.config, layer_id=0, child=layer)
    assert isinstance(cont, C.DS_LLAMAContainer)
    cfg = cont.create_ds_model_config()
    assert cfg.heads == 4 and cfg.num_kv == 2 and cfg.rotate_half and cfg.intermediate_size == 2 * H


@pytest.mark.gpu
@pytest.mark.parametrize("kind,policy", [("llama", "LLAMALayerPolicy"), ("gpt2", "HFGPT2LayerPolicy"),
                                         ("bloom", "BLOOMLayerPolicy")])
def test_hf_layers_replaced_through_policies_gpu(kind, policy):
    """Per-layer injection on the device: the swapped-in layers run the HIP kernels in bf16."""
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.module_inject import containers as C
    m = tiny(kind, H=256).eval()
    ids = torch.randint(0, m.config.vocab_size, (2, 24), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = m(ids, use_cache=False).logits.float()
    eng = ds.init_inference(m, dtype=torch.bfloat16, injection_policy={_layer_cls(kind): getattr(C, policy)})
    assert eng.policy_injected == m.config.num_hidden_layers
    with torch.no_grad():
        out = eng(ids.cuda(), use_cache=False).logits.float().cpu()
    assert (out - ref).abs().max().item() < 0.05 * ref.abs().max().item() + 0.03
