"""Layer policies and containers of the supported client architectures (reference `module_inject/containers/*.py`,
`replace_policy.py`, `utils.py`).

A policy reads one client layer (see `policy.py`); its container turns what the policy returns into one fused
inference layer (`ops/transformer/inference/layer.py: DeepSpeedTransformerInference`, the layer the kernel-injected
engine is made of) and loads this rank's slice of the weights. `init_inference(model, injection_policy={Layer:
Policy})` swaps every `Layer` instance for the container's module. Whole-model injection of the Hugging Face
families (`replace_with_kernel_inject=True`) goes through `inference/model_implementations/convert.py`, which shares
the layouts documented here.
"""
import torch
import torch.nn as nn

from ..ops.transformer.inference.config import DeepSpeedInferenceConfig
from ..ops.transformer.inference.layer import DeepSpeedTransformerInference
from ..utils.types import ActivationFuncType, NormType
from .policy import DSPolicy, TransformerPolicy, transpose

__path__ = []  # lets the reference's per-architecture sub-paths resolve through `_import_paths`
DEFAULT_INTERMEDIATE_SIZE = -1


def _cat(*ts):
    return None if any(t is None for t in ts) else torch.cat([t.detach() for t in ts], dim=0)


def _d(t):
    return None if t is None else t.detach()


def _interleaved_to_blocks(w, heads):
    """Per-head interleaved fused QKV rows [head, (q, k, v), D] -> [q | k | v]."""
    D = w.shape[0] // (3 * heads)
    g = w.reshape(heads, 3, D, *w.shape[1:])
    return torch.cat([g[:, i].reshape(heads * D, *w.shape[1:]) for i in range(3)], dim=0)


# ------------------------------------------------------------------------------------------------ decoder policies
class _Decoder(TransformerPolicy):
    """Shared plumbing: subclasses name the sub-modules."""

    def __init__(self, client_module, inference=True, **kw):
        super().__init__(inference, **kw)
        self.client_module = client_module


class HFGPT2LayerPolicy(_Decoder):
    _orig_layer_class = None

    def __init__(self, client_module, inference=True):
        super().__init__(client_module, inference, linear_layer=False)   # Conv1D weights
        try:
            import transformers
            HFGPT2LayerPolicy._orig_layer_class = transformers.models.gpt2.modeling_gpt2.GPT2Block
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.attn
        return a.embed_dim, a.num_heads, self.client_module.ln_1.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.attn
        return transpose(a.c_attn.weight), _d(a.c_attn.bias), transpose(a.c_proj.weight), _d(a.c_proj.bias)

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return transpose(m.c_fc.weight), _d(m.c_fc.bias), transpose(m.c_proj.weight), _d(m.c_proj.bias)

    def layernorm(self):
        c = self.client_module
        return c.ln_2.weight, c.ln_2.bias, c.ln_1.weight, c.ln_1.bias


class HFGPTJLayerPolicy(_Decoder):
    _orig_layer_class = None

    def __init__(self, client_module, inference=True):
        super().__init__(client_module, inference, scale_attention=True)
        self.mlp_after_attn = False          # parallel attention + MLP off one LayerNorm
        self.rotate_every_two = True
        self.rotary_dim = getattr(client_module.attn, "rotary_dim", None) or -1
        self.return_tuple = True        # GPTJModel indexes the block's output
        try:
            import transformers
            HFGPTJLayerPolicy._orig_layer_class = transformers.models.gptj.modeling_gptj.GPTJBlock
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.attn
        return a.embed_dim, a.num_attention_heads, self.client_module.ln_1.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.attn
        return _cat(a.q_proj.weight, a.k_proj.weight, a.v_proj.weight), None, _d(a.out_proj.weight), None

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return _d(m.fc_in.weight), _d(m.fc_in.bias), _d(m.fc_out.weight), _d(m.fc_out.bias)

    def layernorm(self):
        c = self.client_module
        return None, None, c.ln_1.weight, c.ln_1.bias


class HFGPTNEOLayerPolicy(_Decoder):
    _orig_layer_class = None

    def __init__(self, client_module, inference=True):
        super().__init__(client_module, inference, scale_attention=False)
        att = client_module.attn.attention
        window = getattr(att, "window_size", None) or getattr(getattr(att, "config", None), "window_size", 0)
        self.window_size = window if getattr(att, "attention_type", "global") == "local" else 0
        self.return_tuple = True        # GPTNeoModel indexes the block's output
        try:
            import transformers
            HFGPTNEOLayerPolicy._orig_layer_class = transformers.models.gpt_neo.modeling_gpt_neo.GPTNeoBlock
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.attn.attention
        return a.embed_dim, a.num_heads, self.client_module.ln_1.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.attn.attention
        return _cat(a.q_proj.weight, a.k_proj.weight, a.v_proj.weight), None, _d(a.out_proj.weight), \
            _d(a.out_proj.bias)

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return _d(m.c_fc.weight), _d(m.c_fc.bias), _d(m.c_proj.weight), _d(m.c_proj.bias)

    def layernorm(self):
        c = self.client_module
        return c.ln_2.weight, c.ln_2.bias, c.ln_1.weight, c.ln_1.bias


class GPTNEOXLayerPolicy(_Decoder):
    _orig_layer_class = None
    version = 0

    def __init__(self, client_module, inference=True, megatron_v2=True, split_qkv=False):
        super().__init__(client_module, inference, megatron_v2=megatron_v2, split_qkv=split_qkv)
        self.mlp_after_attn = False
        self.rotate_half = True
        att = client_module.attention
        self.rotary_dim = getattr(att, "rotary_ndims", None) or getattr(att, "head_size", -1)
        cfg = getattr(att, "config", None)
        rp = getattr(cfg, "rope_parameters", None) or {}
        self.rope_theta = float((rp.get("rope_theta") if isinstance(rp, dict) else None)
                                or getattr(cfg, "rotary_emb_base", 10000.0))
        if cfg is not None and not getattr(cfg, "use_parallel_residual", True):
            self.mlp_after_attn = True
        try:
            import transformers
            GPTNEOXLayerPolicy._orig_layer_class = transformers.models.gpt_neox.modeling_gpt_neox.GPTNeoXLayer
        except ImportError:
            pass

    def _heads(self):
        att = self.client_module.attention
        return getattr(att, "num_attention_heads", None) or att.config.num_attention_heads

    def get_hidden_heads(self):
        att = self.client_module.attention
        return att.query_key_value.weight.shape[1], self._heads(), self.client_module.input_layernorm.eps, \
            DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        att = self.client_module.attention
        h = self._heads()
        return _interleaved_to_blocks(att.query_key_value.weight.detach(), h), \
            _interleaved_to_blocks(att.query_key_value.bias.detach(), h), _d(att.dense.weight), _d(att.dense.bias)

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return _d(m.dense_h_to_4h.weight), _d(m.dense_h_to_4h.bias), _d(m.dense_4h_to_h.weight), \
            _d(m.dense_4h_to_h.bias)

    def layernorm(self):
        c = self.client_module
        return c.post_attention_layernorm.weight, c.post_attention_layernorm.bias, c.input_layernorm.weight, \
            c.input_layernorm.bias


class HFOPTLayerPolicy(_Decoder):
    _orig_layer_class = None

    def __init__(self, client_module, inference=True, use_load_prefix=True):
        super().__init__(client_module, inference, linear_layer=True, pre_attn_norm=True,
                         use_load_prefix=use_load_prefix, mlp_act_func_type=ActivationFuncType.ReLU)
        try:
            import transformers
            HFOPTLayerPolicy._orig_layer_class = transformers.models.opt.modeling_opt.OPTDecoderLayer
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.self_attn
        return a.embed_dim, a.num_heads, self.client_module.self_attn_layer_norm.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.self_attn
        return _cat(a.q_proj.weight, a.k_proj.weight, a.v_proj.weight), \
            _cat(a.q_proj.bias, a.k_proj.bias, a.v_proj.bias), _d(a.out_proj.weight), _d(a.out_proj.bias)

    def mlp(self, enable_training=False):
        c = self.client_module
        return _d(c.fc1.weight), _d(c.fc1.bias), _d(c.fc2.weight), _d(c.fc2.bias)

    def layernorm(self):
        c = self.client_module
        return c.final_layer_norm.weight, c.final_layer_norm.bias, c.self_attn_layer_norm.weight, \
            c.self_attn_layer_norm.bias


class BLOOMLayerPolicy(_Decoder):
    _orig_layer_class = None

    def __init__(self, client_module, inference=True, use_load_prefix=True, split_qkv=False):
        super().__init__(client_module, inference, linear_layer=True, use_load_prefix=use_load_prefix,
                         split_qkv=split_qkv)
        self.bigscience_bloom = True
        self.return_tuple = True        # BloomModel indexes the block's output
        try:
            import transformers
            BLOOMLayerPolicy._orig_layer_class = transformers.models.bloom.modeling_bloom.BloomBlock
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.self_attention
        return a.hidden_size, a.num_heads, self.client_module.input_layernorm.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.self_attention
        h = a.num_heads
        return _interleaved_to_blocks(a.query_key_value.weight.detach(), h), \
            _interleaved_to_blocks(a.query_key_value.bias.detach(), h), _d(a.dense.weight), _d(a.dense.bias)

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return _d(m.dense_h_to_4h.weight), _d(m.dense_h_to_4h.bias), _d(m.dense_4h_to_h.weight), \
            _d(m.dense_4h_to_h.bias)

    def layernorm(self):
        c = self.client_module
        return c.post_attention_layernorm.weight, c.post_attention_layernorm.bias, c.input_layernorm.weight, \
            c.input_layernorm.bias


class LLAMALayerPolicy(_Decoder):
    """Hugging Face Llama-family decoder layer (RMSNorm, rotate-half RoPE, gated SiLU MLP, grouped KV heads)."""
    _orig_layer_class = None

    def __init__(self, client_module, inference=True):
        super().__init__(client_module, inference, mlp_act_func_type=ActivationFuncType.GATED_SILU,
                         norm_type=NormType.RMSNorm)
        a = client_module.self_attn
        cfg = getattr(a, "config", None)
        self.rotate_half = True
        self.rotary_dim = getattr(a, "head_dim", None) or (cfg.hidden_size // cfg.num_attention_heads)
        self.num_kv = getattr(cfg, "num_key_value_heads", None) or getattr(a, "num_key_value_heads", -1)
        rp = getattr(cfg, "rope_parameters", None) or {}
        self.rope_theta = float((rp.get("rope_theta") if isinstance(rp, dict) else None)
                                or getattr(cfg, "rope_theta", 10000.0))
        try:
            import transformers
            LLAMALayerPolicy._orig_layer_class = transformers.models.llama.modeling_llama.LlamaDecoderLayer
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.self_attn
        cfg = a.config
        return cfg.hidden_size, cfg.num_attention_heads, self.client_module.input_layernorm.variance_epsilon, \
            self.client_module.mlp.gate_proj.weight.shape[0]

    def attention(self, enable_training=False):
        a = self.client_module.self_attn
        return _cat(a.q_proj.weight, a.k_proj.weight, a.v_proj.weight), \
            _cat(a.q_proj.bias, a.k_proj.bias, a.v_proj.bias) if a.q_proj.bias is not None else None, \
            _d(a.o_proj.weight), _d(a.o_proj.bias)

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return _cat(m.gate_proj.weight, m.up_proj.weight), None, _d(m.down_proj.weight), None

    def layernorm(self):
        c = self.client_module
        return c.post_attention_layernorm.weight, None, c.input_layernorm.weight, None


class InternLMLayerPolicy(LLAMALayerPolicy):
    """InternLM: the Llama layer with biased attention projections."""


class LLAMA2LayerPolicy(_Decoder):
    """Meta's own Llama-2 `TransformerBlock` (attention.wq / wk / wv / wo, feed_forward.w1 / w3 / w2)."""
    _orig_layer_class = None

    def __init__(self, client_module, inference=True):
        super().__init__(client_module, inference, mlp_act_func_type=ActivationFuncType.GATED_SILU,
                         norm_type=NormType.RMSNorm)
        a = client_module.attention
        self.rotate_every_two = True            # Meta's checkpoints rotate (x[2i], x[2i+1]) pairs
        self.rotary_dim = a.wq.weight.shape[0] // getattr(a, "n_local_heads", getattr(a, "n_heads", 1))
        self.num_kv = getattr(a, "n_local_kv_heads", getattr(a, "n_kv_heads", -1))

    def get_hidden_heads(self):
        a = self.client_module.attention
        heads = getattr(a, "n_local_heads", None) or a.n_heads
        return a.wq.weight.shape[1], heads, self.client_module.ffn_norm.eps, \
            self.client_module.feed_forward.w1.weight.shape[0]

    def attention(self, enable_training=False):
        a = self.client_module.attention
        return _cat(a.wq.weight, a.wk.weight, a.wv.weight), None, _d(a.wo.weight), None

    def mlp(self, enable_training=False):
        f = self.client_module.feed_forward
        return _cat(f.w1.weight, f.w3.weight), None, _d(f.w2.weight), None

    def layernorm(self):
        c = self.client_module
        return c.ffn_norm.weight, None, c.attention_norm.weight, None


class MegatronLayerPolicy(_Decoder):
    """Megatron-LM GPT `ParallelTransformerLayer` (fused query_key_value, head-interleaved from v2 on)."""
    _orig_layer_class = None
    version = 0
    moe_type = "standard"
    megatron_v2 = True
    use_mup = False

    def __init__(self, client_module, inference=True):
        super().__init__(client_module, inference, megatron_v2=MegatronLayerPolicy.megatron_v2,
                         use_mup=MegatronLayerPolicy.use_mup)

    def _attn(self):
        c = self.client_module
        return c.attention if hasattr(c, "attention") else c.self_attention

    def get_hidden_heads(self):
        a = self._attn()
        heads = getattr(a, "num_attention_heads", None) or a.num_attention_heads_per_partition
        return a.query_key_value.weight.shape[1], heads, self.client_module.input_layernorm.eps, \
            DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self._attn()
        w, b = a.query_key_value.weight.detach(), a.query_key_value.bias.detach()
        if self.is_megatron_v2:
            h = self.get_hidden_heads()[1]
            w, b = _interleaved_to_blocks(w, h), _interleaved_to_blocks(b, h)
        return w, b, _d(a.dense.weight), _d(a.dense.bias)

    def mlp(self, moe_type="standard", enable_training=False):
        m = self.client_module.mlp
        return _d(m.dense_h_to_4h.weight), _d(m.dense_h_to_4h.bias), _d(m.dense_4h_to_h.weight), \
            _d(m.dense_4h_to_h.bias)

    def layernorm(self):
        c = self.client_module
        return c.post_attention_layernorm.weight, c.post_attention_layernorm.bias, c.input_layernorm.weight, \
            c.input_layernorm.bias


class MegatronMoELayerPolicy(MegatronLayerPolicy):
    """Megatron GPT-MoE layer: `mlp.deepspeed_moe.experts.deepspeed_experts[i]` dense experts (standard), or
    `mlp.moe.deepspeed_moe` + `mlp.mlp` + `mlp.coefficient` (residual MoE)."""
    num_experts = 1

    def get_num_experts(self):
        return self.num_experts

    def mlp(self, moe_type="standard", enable_training=False):
        m = self.client_module.mlp
        moe = m.deepspeed_moe if moe_type == "standard" else m.moe.deepspeed_moe
        ex = moe.experts.deepspeed_experts
        self.num_experts = len(ex)
        out = ([e.dense_h_to_4h.weight.detach() for e in ex], [e.dense_h_to_4h.bias.detach() for e in ex],
               [e.dense_4h_to_h.weight.detach() for e in ex], [e.dense_4h_to_h.bias.detach() for e in ex])
        if moe_type == "standard":
            return out
        return out + (_d(m.mlp.dense_h_to_4h.weight), _d(m.mlp.dense_h_to_4h.bias), _d(m.mlp.dense_4h_to_h.weight),
                      _d(m.mlp.dense_4h_to_h.bias), _d(m.coefficient.weight))


# ------------------------------------------------------------------------------------------------ encoder policies
class HFBertLayerPolicy(TransformerPolicy):
    _orig_layer_class = None

    def __init__(self, client_module, inference=False):
        super().__init__(inference, pre_attn_norm=False)
        self.client_module = client_module
        self.cuda_graph_supported = True
        try:
            import transformers
            HFBertLayerPolicy._orig_layer_class = [transformers.models.bert.modeling_bert.BertLayer,
                                                   transformers.models.roberta.modeling_roberta.RobertaLayer]
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.attention
        ln = a.output.LayerNorm
        return a.self.query.weight.shape[1], a.self.num_attention_heads, ln.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        s, o = self.client_module.attention.self, self.client_module.attention.output
        return _cat(s.query.weight, s.key.weight, s.value.weight), _cat(s.query.bias, s.key.bias, s.value.bias), \
            _d(o.dense.weight), _d(o.dense.bias)

    def mlp(self, enable_training=False):
        c = self.client_module
        return _d(c.intermediate.dense.weight), _d(c.intermediate.dense.bias), _d(c.output.dense.weight), \
            _d(c.output.dense.bias)

    def layernorm(self):
        c = self.client_module
        a, t = c.attention.output.LayerNorm, c.output.LayerNorm
        return a.weight, a.bias, t.weight, t.bias


class HFDistilBertLayerPolicy(TransformerPolicy):
    _orig_layer_class = None

    def __init__(self, client_module, inference=False, preln=False):
        super().__init__(inference, pre_attn_norm=preln)
        self.client_module = client_module
        self.cuda_graph_supported = True
        try:
            import transformers
            HFDistilBertLayerPolicy._orig_layer_class = \
                transformers.models.distilbert.modeling_distilbert.TransformerBlock
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.attention
        return a.q_lin.weight.shape[1], a.n_heads, self.client_module.sa_layer_norm.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.attention
        return _cat(a.q_lin.weight, a.k_lin.weight, a.v_lin.weight), _cat(a.q_lin.bias, a.k_lin.bias, a.v_lin.bias), \
            _d(a.out_lin.weight), _d(a.out_lin.bias)

    def mlp(self, enable_training=False):
        f = self.client_module.ffn
        return _d(f.lin1.weight), _d(f.lin1.bias), _d(f.lin2.weight), _d(f.lin2.bias)

    def layernorm(self):
        c = self.client_module
        return c.sa_layer_norm.weight, c.sa_layer_norm.bias, c.output_layer_norm.weight, c.output_layer_norm.bias


class HFCLIPLayerPolicy(TransformerPolicy):
    _orig_layer_class = None

    def __init__(self, client_module, inference=False):
        super().__init__(inference, pre_attn_norm=True, scale_attention=True)
        self.client_module = client_module
        self.cuda_graph_supported = True
        try:
            import transformers
            HFCLIPLayerPolicy._orig_layer_class = transformers.models.clip.modeling_clip.CLIPEncoderLayer
        except ImportError:
            pass

    def get_hidden_heads(self):
        a = self.client_module.self_attn
        return a.q_proj.weight.shape[1], a.num_heads, self.client_module.layer_norm1.eps, DEFAULT_INTERMEDIATE_SIZE

    def attention(self, enable_training=False):
        a = self.client_module.self_attn
        return _cat(a.q_proj.weight, a.k_proj.weight, a.v_proj.weight), \
            _cat(a.q_proj.bias, a.k_proj.bias, a.v_proj.bias), _d(a.out_proj.weight), _d(a.out_proj.bias)

    def mlp(self, enable_training=False):
        m = self.client_module.mlp
        return _d(m.fc1.weight), _d(m.fc1.bias), _d(m.fc2.weight), _d(m.fc2.bias)

    def layernorm(self):
        c = self.client_module
        return c.layer_norm2.weight, c.layer_norm2.bias, c.layer_norm1.weight, c.layer_norm1.bias


# ------------------------------------------------------------------------------------------------ diffusers policies
class UNetPolicy(DSPolicy):

    def __init__(self):
        super().__init__()
        try:
            import diffusers
            self._orig_layer_class = diffusers.models.unet_2d_condition.UNet2DConditionModel
        except Exception:
            self._orig_layer_class = None

    def match(self, module):
        return type(module).__name__ == "UNet2DConditionModel"

    def match_replaced(self, module):
        from .diffusers import DSUNet
        return isinstance(module, DSUNet)

    def apply(self, module, enable_cuda_graph=True):
        from .diffusers import DSUNet
        return DSUNet(module, enable_cuda_graph=enable_cuda_graph)

    def attention(self, client_module):
        """(qkv weight or None, q, k, v weights, output weight, output bias, heads) of a diffusers attention."""
        qw, kw, vw = client_module.to_q.weight, client_module.to_k.weight, client_module.to_v.weight
        ow, ob = client_module.to_out[0].weight, client_module.to_out[0].bias
        heads = client_module.heads
        if qw.shape[1] == kw.shape[1]:      # self attention: fuse
            return torch.cat([qw, kw, vw], dim=0).detach(), None, None, None, _d(ow), _d(ob), heads
        return None, _d(qw), _d(kw), _d(vw), _d(ow), _d(ob), heads


class VAEPolicy(DSPolicy):

    def __init__(self):
        super().__init__()
        try:
            import diffusers
            self._orig_layer_class = diffusers.models.autoencoder_kl.AutoencoderKL
        except Exception:
            self._orig_layer_class = None

    def match(self, module):
        return type(module).__name__ == "AutoencoderKL"

    def match_replaced(self, module):
        from .diffusers import DSVAE
        return isinstance(module, DSVAE)

    def apply(self, module, enable_cuda_graph=True):
        from .diffusers import DSVAE
        return DSVAE(module, enable_cuda_graph=enable_cuda_graph)

    def attention(self, client_module):
        return None


# ------------------------------------------------------------------------------------------------ containers
class _InjectedLayer(nn.Module):
    """The fused layer behind a client layer's call signature: first positional argument (or `hidden_states`) in,
    hidden states out — a tensor, or a 1-tuple when the policy says the client returned tuples."""

    def __init__(self, ds_layer, return_tuple):
        super().__init__()
        self.ds_layer = ds_layer
        self.return_tuple = return_tuple

    def forward(self, *args, **kwargs):
        h = args[0] if args else kwargs.get("hidden_states", kwargs.get("x"))
        past = kwargs.get("layer_past")
        out = self.ds_layer(h, layer_past=past)
        out = out[0] if isinstance(out, tuple) else out
        return (out, ) if self.return_tuple else out


class BaseTransformerContainer:
    """policy -> `DeepSpeedInferenceConfig` -> fused layer with this rank's weights (reference
    `containers/base.py:BaseTransformerContainer`)."""

    def __init__(self, policy, config=None, model_config=None, layer_id=0, child=None):
        self.policy, self.config, self.model_config, self.layer_id, self.child = policy, config, model_config, \
            layer_id, child
        self.hidden_size, self.num_attention_heads, self.layernorm_epsilon, self.intermediate_size = \
            policy.get_hidden_heads()
        self.mp_size = config.tensor_parallel.tp_size if config is not None else 1
        self.mp_group = config.tensor_parallel.tp_group if config is not None else None
        self.dtype = (config.dtype if config is not None else None) or torch.bfloat16
        self.max_out_tokens = getattr(config, "max_out_tokens", 1024) if config is not None else 1024
        self.module = None
        self.ds_model_config = None

    # -- step 1
    def create_ds_model_config(self):
        p = self.policy
        self.initialize_tensors()
        inter = self.intermediate_size
        if inter is None or inter <= 0:
            rows = self._inter_w.shape[0]
            inter = rows // 2 if p.mlp_act_func_type in (ActivationFuncType.GATED_SILU,
                                                         ActivationFuncType.GATED_GELU) else rows
        self.ds_model_config = DeepSpeedInferenceConfig(
            hidden_size=self.hidden_size, intermediate_size=inter, heads=self.num_attention_heads,
            layer_norm_eps=self.layernorm_epsilon, mp_size=self.mp_size, dtype=self.dtype,
            pre_layer_norm=p.pre_attn_norm, norm_type=p.norm_type, scale_attention=p.scale_attention,
            local_attention=bool(p.window_size), window_size=p.window_size or 256, rotary_dim=p.rotary_dim,
            rotate_half=p.rotate_half, rotate_every_two=p.rotate_every_two, return_tuple=p.return_tuple,
            mlp_after_attn=p.mlp_after_attn, mlp_act_func_type=p.mlp_act_func_type,
            bigscience_bloom=p.bigscience_bloom, max_out_tokens=self.max_out_tokens, num_kv=p.num_kv,
            rope_theta=p.rope_theta)
        # a parallel block whose policy returns no second norm runs both branches off the input norm (GPT-J)
        self.ds_model_config.shared_parallel_norm = self._attn_nw is None
        return self.ds_model_config

    def initialize_tensors(self, enable_training=False):
        self._qkvw, self._qkvb, self._dense_w, self._dense_b = self.policy.attention()
        self._inter_w, self._inter_b, self._out_w, self._out_b = self.policy.mlp()[:4]
        self._attn_nw, self._attn_nb, self._input_nw, self._input_nb = self.policy.layernorm()

    # -- step 2
    def create_module(self, config=None):
        cfg = config or self.ds_model_config or self.create_ds_model_config()
        device = self._qkvw.device if self._qkvw.device.type != "meta" else None
        self.module = DeepSpeedTransformerInference(cfg, mp_group=self.mp_group, device=device)
        return self.module

    # -- step 3
    def apply_tensor_parallelism(self, mp_replace=None):
        """This rank's slices (query heads / kv heads / intermediate rows), done when the weights are copied."""
        return None

    def copy_data_to_new_module(self):
        from ..inference.v2.model_implementations import sharding as S
        tp = self.mp_size if self.mp_group is not None else 1
        rank = 0
        if tp > 1:
            from .. import comm as dist
            rank = dist.get_rank(self.mp_group)
        heads = self.num_attention_heads
        hd = self.hidden_size // heads
        nkv = self.policy.num_kv if self.policy.num_kv and self.policy.num_kv > 0 else heads
        gated = self.policy.mlp_act_func_type in (ActivationFuncType.GATED_SILU, ActivationFuncType.GATED_GELU)
        qkvw = S.shard_qkv_param(self._qkvw, rank, tp, hd, heads, nkv)
        qkvb = S.shard_qkv_param(self._qkvb, rank, tp, hd, heads, nkv)
        ow = S.shard_attn_out_param(self._dense_w, rank, tp, hd, heads, nkv)
        inter_w = S.shard_mlp_1_param(self._inter_w, rank, tp, gated=gated)
        inter_b = S.shard_mlp_1_param(self._inter_b, rank, tp, gated=gated)
        out_w = S.shard_mlp_2_param(self._out_w, rank, tp)
        self.module.load_weights(qkvw, ow, inter_w, out_w, attn_nw=self._input_nw, norm_w=self._attn_nw,
                                 attn_qkvb=qkvb, attn_ob=self._dense_b, inter_b=inter_b, output_b=self._out_b,
                                 attn_nb=self._input_nb, norm_b=self._attn_nb)
        return self.module

    def build(self):
        """All steps: the module to put where the client layer was."""
        self.create_ds_model_config()
        self.create_module()
        self.copy_data_to_new_module()
        return _InjectedLayer(self.module, self.policy.return_tuple)


class BaseTransformerMoEContainer(BaseTransformerContainer):
    """MoE client layers are injected whole-model (`convert._megatron_gpt`, `_mixtral`): the per-layer container
    only reads the experts through its policy."""

    def initialize_tensors(self, enable_training=False):
        self._qkvw, self._qkvb, self._dense_w, self._dense_b = self.policy.attention()
        self._attn_nw, self._attn_nb, self._input_nw, self._input_nb = self.policy.layernorm()
        self.experts = self.policy.mlp(getattr(self.policy, "moe_type", "standard"))
        self._inter_w, self._inter_b, self._out_w, self._out_b = (t[0] for t in self.experts[:4])

    def build(self):
        raise NotImplementedError("expert layers are injected through init_inference(replace_with_kernel_inject="
                                  "True) on the whole model")


class BaseConvolutionContainer:
    """Diffusers UNet / VAE: whole-module wrappers (graph capture + fused attention), see `diffusers.py`."""


def _container(name, policy_doc):
    return type(name, (BaseTransformerContainer, ), {"__doc__": policy_doc})


DS_GPT2Container = _container("DS_GPT2Container", "GPT-2 block (Conv1D weights transposed on read).")
DS_GPTJContainer = _container("DS_GPTJContainer", "GPT-J block (parallel MLP, interleaved RoPE).")
DS_GPTNEOContainer = _container("DS_GPTNEOContainer", "GPT-Neo block (unscaled scores, local attention layers).")
DS_GPTNEOXContainer = _container("DS_GPTNEOXContainer", "GPT-NeoX layer (interleaved fused QKV, parallel MLP).")
DS_OPTContainer = _container("DS_OPTContainer", "OPT decoder layer (ReLU MLP).")
DS_BloomContainer = _container("DS_BloomContainer", "BLOOM block (ALiBi, interleaved fused QKV).")
DS_LLAMAContainer = _container("DS_LLAMAContainer", "HF Llama decoder layer.")
DS_LLAMA2Container = _container("DS_LLAMA2Container", "Meta Llama-2 TransformerBlock.")
DS_InternLMContainer = _container("DS_InternLMContainer", "InternLM decoder layer.")
DS_MegatronGPTContainer = _container("DS_MegatronGPTContainer", "Megatron-LM GPT layer.")
DS_MegatronGPTMoEContainer = type("DS_MegatronGPTMoEContainer", (BaseTransformerMoEContainer, ), {})


class _EncoderContainer(BaseTransformerContainer):
    """Bidirectional encoder layers run on `module_inject/encoder.py: DSEncoderLayer`."""

    def build(self):
        from . import encoder as enc
        for pred, make in ((enc._is_bert_layer, enc._from_bert), (enc._is_distil_block, enc._from_distil),
                           (enc._is_clip_layer, enc._from_clip)):
            if pred(self.policy.client_module):
                cfg = self.model_config
                return make(self.policy.client_module, cfg, tp_group=self.mp_group, tp_size=self.mp_size,
                            tp_rank=0, dtype=self.dtype, device=next(self.policy.client_module.parameters()).device)
        raise NotImplementedError(f"no encoder layer builder for {type(self.policy.client_module).__name__}")


DS_BERTContainer = type("DS_BERTContainer", (_EncoderContainer, ), {})
DS_DistilBERTContainer = type("DS_DistilBERTContainer", (_EncoderContainer, ), {})
DS_CLIPContainer = type("DS_CLIPContainer", (_EncoderContainer, ), {})

supported_models = {None}   # BLOOM container's model registry in the reference (filled from transformers when present)
try:
    import transformers as _tf
    supported_models = {_tf.models.bloom.modeling_bloom.BloomModel}
except Exception:
    pass

# policy -> container
_CONTAINERS = {
    HFGPT2LayerPolicy: DS_GPT2Container, HFGPTJLayerPolicy: DS_GPTJContainer, HFGPTNEOLayerPolicy: DS_GPTNEOContainer,
    GPTNEOXLayerPolicy: DS_GPTNEOXContainer, HFOPTLayerPolicy: DS_OPTContainer, BLOOMLayerPolicy: DS_BloomContainer,
    LLAMALayerPolicy: DS_LLAMAContainer, LLAMA2LayerPolicy: DS_LLAMA2Container,
    InternLMLayerPolicy: DS_InternLMContainer, MegatronLayerPolicy: DS_MegatronGPTContainer,
    MegatronMoELayerPolicy: DS_MegatronGPTMoEContainer, HFBertLayerPolicy: DS_BERTContainer,
    HFDistilBertLayerPolicy: DS_DistilBERTContainer, HFCLIPLayerPolicy: DS_CLIPContainer,
}

replace_policies = [HFBertLayerPolicy, HFGPTNEOLayerPolicy, GPTNEOXLayerPolicy, HFGPTJLayerPolicy,
                    MegatronLayerPolicy, HFGPT2LayerPolicy, BLOOMLayerPolicy, HFOPTLayerPolicy, HFCLIPLayerPolicy,
                    HFDistilBertLayerPolicy, LLAMALayerPolicy, LLAMA2LayerPolicy, InternLMLayerPolicy]
generic_policies = [UNetPolicy, VAEPolicy]


def policy_to_ds_container(**kwargs):
    """Container instance for `policy=` (reference `module_inject/utils.py`); other keywords go to the container."""
    policy = kwargs["policy"]
    for cls in type(policy).__mro__:
        if cls in _CONTAINERS:
            return _CONTAINERS[cls](**kwargs)
    if isinstance(policy, TransformerPolicy):     # a user-defined policy: the generic container
        return BaseTransformerContainer(**kwargs)
    raise ValueError(f"no container for policy {type(policy).__name__}")


def replace_layers_with_policy(model, layer_class, policy_class, config=None, model_config=None):
    """Swap every `layer_class` instance of `model` for the fused layer its policy describes. Returns the count."""
    n = 0
    for name, child in list(model.named_modules()):
        if not isinstance(child, layer_class) or not name:
            continue
        policy = policy_class(child)
        fused = policy_to_ds_container(policy=policy, config=config, model_config=model_config, layer_id=n,
                                       child=child).build()
        parent_name, _, leaf = name.rpartition(".")
        parent = model.get_submodule(parent_name) if parent_name else model
        setattr(parent, leaf, fused)
        n += 1
    return n
