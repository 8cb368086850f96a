"""Container feature mixins (`module_inject/container_features.py`; reference
`module_inject/containers/features/*.py`): meta-device layers filled from a state dict, Megatron v2 QKV re-layout,
and the per-layer hybrid-engine switches (LoRA folding, release / reset of the inference copy)."""
import torch
import torch.nn as nn

from .test_layer_policies import _Block


def _policy_cls():
    from deepspeedsyclsupport_amd.module_inject.policy import TransformerPolicy
    from deepspeedsyclsupport_amd.utils.types import ActivationFuncType

    class BlockPolicy(TransformerPolicy):

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

    return BlockPolicy


class _Cfg:
    """The parts of an inference config a container reads."""

    class tensor_parallel:
        tp_size, tp_group = 1, None

    dtype = torch.float32
    max_out_tokens = 64


def test_meta_tensor_container_loads_from_state_dict():
    from deepspeedsyclsupport_amd.module_inject import containers as C
    from deepspeedsyclsupport_amd.module_inject.container_features import MetaTensorContainer

    class Cont(MetaTensorContainer, C.BaseTransformerContainer):
        pass

    torch.manual_seed(0)
    real = _Block().eval()
    sd = {"layers.3." + k: v for k, v in real.state_dict().items()}
    with torch.device("meta"):
        ghost = _Block()
    cont = Cont(policy=_policy_cls()(ghost), config=_Cfg, layer_id=0)
    cont.create_ds_model_config()
    assert cont.is_meta
    cont.create_module()
    assert cont.copy_data_to_new_module() is cont.module      # nothing to copy yet
    cont.load_params(sd=[sd], prefix="layers.3.")
    assert not cont.is_meta and not any(p.is_meta for p in ghost.parameters())
    x = torch.randn(2, 7, 64)
    with torch.no_grad():
        out = cont.module(x)
        out = out[0] if isinstance(out, tuple) else out
        torch.testing.assert_close(out, real(x), rtol=1e-4, atol=1e-4)
    try:
        with torch.device("meta"):
            g2 = _Block()
        c2 = Cont(policy=_policy_cls()(g2), config=_Cfg, layer_id=1)
        c2.create_ds_model_config()
        c2.load_params(sd=sd, prefix="nowhere.")
    except KeyError as e:
        assert "nowhere." in str(e)
    else:
        raise AssertionError("a checkpoint without the layer's keys must raise")


def test_megatron_v2_alignment_roundtrip():
    from deepspeedsyclsupport_amd.module_inject import containers as C
    from deepspeedsyclsupport_amd.module_inject.container_features import HybridMegatronContainer

    class Cont(HybridMegatronContainer, C.BaseTransformerContainer):
        pass

    blk = _Block()
    pol = _policy_cls()(blk)
    pol.is_megatron_v2 = True
    cont = Cont(policy=pol, config=_Cfg, layer_id=0)
    heads, hd = 4, 16
    w = torch.arange(3 * 64, dtype=torch.float32)[:, None].repeat(1, 2)       # row index in column 0
    aligned = cont._align_qkv(w)
    # row (head h, part p, d) moves to block p, row h*hd + d
    h, p, d = 2, 1, 5
    assert aligned[p * 64 + h * hd + d, 0] == (h * 3 + p) * hd + d
    torch.testing.assert_close(cont._partition_qkv(aligned), w)
    cont.initialize_tensors()
    before = cont._qkvw.clone()
    cont.transpose()
    torch.testing.assert_close(cont._qkvw, cont._align_qkv(before))


class _LoRALinear(nn.Linear):

    def __init__(self, i, o, r=4):
        super().__init__(i, o)
        self.lora_right_weight = nn.Parameter(torch.randn(i, r) * 0.1)
        self.lora_left_weight = nn.Parameter(torch.randn(r, o) * 0.1)
        self.lora_scaling = 0.5

    def forward(self, x):
        return super().forward(x) + self.lora_scaling * (x @ self.lora_right_weight @ self.lora_left_weight)


def test_hybrid_container_lora_release_reset():
    from deepspeedsyclsupport_amd.module_inject import containers as C
    from deepspeedsyclsupport_amd.module_inject.container_features import HybridEngineContainer

    class Cont(HybridEngineContainer, C.BaseTransformerContainer):
        pass

    torch.manual_seed(1)
    blk = _Block().eval()
    blk.wo = _LoRALinear(64, 64)
    blk.b = _LoRALinear(128, 64)
    cont = Cont(policy=_policy_cls()(blk), config=_Cfg, layer_id=0)
    cont.create_ds_model_config()
    assert len(cont.lora_params) == 2 and len(cont.get_lora_params()) == 2
    w0 = blk.wo.weight.detach().clone()
    cont.transform_for_inference()                      # folds LoRA into the fused copy, leaves the client as it was
    torch.testing.assert_close(blk.wo.weight, w0)
    x = torch.randn(2, 5, 64)

    def fused(x):
        with torch.no_grad():
            o = cont.module(x)
        return o[0] if isinstance(o, tuple) else o

    with torch.no_grad():
        ref = blk(x)
    torch.testing.assert_close(fused(x), ref, rtol=1e-4, atol=1e-4)
    # a "training step", then the switch picks the new weights up
    with torch.no_grad():
        blk.a.weight.mul_(1.1)
        blk.wo.lora_left_weight.add_(0.05)
        ref2 = blk(x)
    assert not torch.allclose(ref, ref2, atol=1e-4)
    cont.transform_for_inference()
    torch.testing.assert_close(fused(x), ref2, rtol=1e-4, atol=1e-4)
    # release drops the inference copy; reset brings it back
    L = cont.module.layer
    held = sum(t.numel() for _, t in cont._fused_tensors())
    cont.release_memory()
    assert sum(t.numel() for _, t in cont._fused_tensors()) == 0 and held > 0 and L.qkv_w.numel() == 0
    cont.fuse_lora()
    cont.reset_params()
    cont.unfuse_lora()
    torch.testing.assert_close(fused(x), ref2, rtol=1e-4, atol=1e-4)
    cont.transform_for_training()
    torch.testing.assert_close(blk.wo.weight, w0)
    # aliasing: the second MLP matrix and the attention output share storage with the client afterwards
    cont.set_params_wo_copy()
    assert L.fc2_w.data_ptr() == blk.b.weight.data_ptr() and L.o_w.data_ptr() == blk.wo.weight.data_ptr()


def test_split_qkv_and_gated_mlp_mixins():
    from deepspeedsyclsupport_amd.module_inject import containers as C
    from deepspeedsyclsupport_amd.module_inject.container_features import (HybridGatedMLPContainer,
                                                                           HybridSplitQKVContainer)
    from .test_inference import tiny
    m = tiny("llama")
    layer = m.model.layers[0]

    class Cont(HybridSplitQKVContainer, HybridGatedMLPContainer, C.DS_LLAMAContainer):

        def set_q_k_v(self):
            a = self.policy.client_module.self_attn
            self.qw, self.kw, self.vw = a.q_proj.weight, a.k_proj.weight, a.v_proj.weight
            self.qb = self.kb = self.vb = None

        def set_mlp_gate(self):
            mlp = self.policy.client_module.mlp
            self.inter_gate_w, self.inter_up_w = mlp.gate_proj.weight, mlp.up_proj.weight
            self.inter_gate_b = self.inter_up_b = None

    cont = Cont(policy=C.LLAMALayerPolicy(layer), config=_Cfg, model_config=m.config, layer_id=0)
    cont.initialize_tensors()
    want_qkv, want_inter = cont._qkvw.clone(), cont._inter_w.clone()
    qkvw, qkvb = cont.attention_qkv_mp()
    iw, ib = cont.mlp_inter_mp()
    torch.testing.assert_close(qkvw, want_qkv)
    torch.testing.assert_close(iw, want_inter)
    assert qkvb is None and ib is None and len(cont.get_attn_params()) == 8 and len(cont.get_mlp_params()) == 6
