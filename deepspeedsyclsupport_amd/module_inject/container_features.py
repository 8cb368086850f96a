"""Optional behaviours of the layer containers, as mixins over `containers.BaseTransformerContainer` (reference
`module_inject/containers/features/{meta_tensor,megatron,hybrid_engine,hybrid_megatron,split_qkv,gated_mlp}.py`).

The fused layer keeps its own copy of the weights in the layouts its kernels want, so "training <-> inference"
for one layer is a re-read of the client's tensors through the policy (`transform_for_inference`), and dropping
the inference copy between generation phases (`release_memory` / `reset_params`) is what frees HBM; the
whole-model counterpart lives in `runtime/hybrid_engine.py`.
"""
import torch

from .containers import _interleaved_to_blocks


class MetaTensorContainer:
    """The client layer was built on the meta device: its weights come from a checkpoint's state dict
    (`load_params`) instead of from the module."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.is_meta = False
        self.ckpt_load_enabled = True

    def initialize_tensors(self, enable_training=False):
        super().initialize_tensors(enable_training=enable_training)
        self.is_meta = self._qkvw.is_meta

    def apply_tensor_parallelism(self, mp_replace=None, **kwargs):
        if self.is_meta:       # nothing to slice yet: `load_params` slices when the weights arrive
            return None
        return super().apply_tensor_parallelism(mp_replace)

    def copy_data_to_new_module(self):
        if self.is_meta:
            return self.module
        return super().copy_data_to_new_module()

    def load_params(self, module=None, sd=None, weight_quantizer=None, mp_replace=None, prefix=""):
        """Materialise the client layer from `sd` (keys `prefix + <name inside the layer>`), then fill the fused
        layer. `sd` may be a list holding one dict, as the reference's loaders pass it."""
        sd = sd[0] if isinstance(sd, (list, tuple)) else sd
        client = self.policy.client_module
        device = self.module.device if self.module is not None and getattr(self.module, "device", None) else "cpu"
        client.to_empty(device=device)
        own = {}
        for name, _ in list(client.named_parameters()) + list(client.named_buffers()):
            if prefix + name in sd:
                own[name] = sd[prefix + name]
        missing, _ = client.load_state_dict(own, strict=False)
        missing = [m for m in missing if m in dict(client.named_parameters())]
        if missing:
            raise KeyError(f"checkpoint has no {prefix}{missing[0]} (and {len(missing) - 1} more)")
        super().initialize_tensors()
        self.is_meta = False
        if self.module is None:
            self.create_module()
        return super().copy_data_to_new_module()


class MegatronContainer:
    """Megatron-LM checkpoints written with the v2 layout store fused QKV per head ([heads, 3, head_dim] rows);
    the fused layer wants [q | k | v] blocks."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.megatron_v2 = getattr(self.policy, "is_megatron_v2", False)

    def _align_qkv_transposed(self, x):
        return None if x is None else _interleaved_to_blocks(x, self.num_attention_heads)

    def transpose(self):
        if self.megatron_v2:
            self._qkvw = self._align_qkv_transposed(self._qkvw)
            self._qkvb = self._align_qkv_transposed(self._qkvb)


class HybridEngineContainer:
    """A layer that trains in the client module and generates in the fused one (RLHF)."""

    def initialize_tensors(self, enable_training=False):
        super().initialize_tensors(enable_training=enable_training)
        self.set_lora_params()

    # ---- LoRA
    def set_lora_params(self):
        """LoRA-wrapped linears of the client layer (modules with `lora_right_weight` / `lora_left_weight` /
        `lora_scaling`, weight [out, in], update = scaling * (right @ left)^T)."""
        self.lora_params = [m for m in self.policy.client_module.modules()
                            if hasattr(m, "lora_right_weight") and hasattr(m, "lora_left_weight")]
        self._lora_fused = False

    def get_lora_params(self):
        return [(m.lora_right_weight, m.lora_left_weight, m.lora_scaling) for m in self.lora_params]

    def get_lora_matched_pair(self):
        """[(base weight, (right, left, scaling))] for every LoRA linear of the layer."""
        return [(m.weight, (m.lora_right_weight, m.lora_left_weight, m.lora_scaling)) for m in self.lora_params]

    def _lora_delta(self, right, left, scaling):
        return scaling * (right @ left).t()

    @torch.no_grad()
    def fuse_lora(self):
        if not self._lora_fused:
            for w, (r, l, s) in self.get_lora_matched_pair():
                w.add_(self._lora_delta(r, l, s).to(w.dtype))
            self._lora_fused = True

    @torch.no_grad()
    def unfuse_lora(self):
        if self._lora_fused:
            for w, (r, l, s) in self.get_lora_matched_pair():
                w.sub_(self._lora_delta(r, l, s).to(w.dtype))
            self._lora_fused = False

    # ---- phase switches
    def transform_for_inference(self):
        """Re-read the (just trained) client tensors into the fused layer, LoRA folded in."""
        self.fuse_lora()
        try:
            super().initialize_tensors()
            if hasattr(self, "transpose"):
                self.transpose()
            if self.module is None:
                self.create_module()
            elif self._released:
                self.reset_params()
                return
            self.copy_data_to_new_module()
        finally:
            self.unfuse_lora()

    def transform_for_training(self):
        """The client module owns the trainable tensors throughout: only a still-fused LoRA has to come out."""
        self.unfuse_lora()

    # ---- memory
    _released = False

    def _fused_tensors(self):
        L = self.module.layer
        return [(n, getattr(L, n)) for n in ("qkv_w", "o_w", "fc1_w", "fc2_w", "qkv_b", "o_b", "fc1_b", "fc2_b")
                if getattr(L, n, None) is not None]

    def release_qkv(self):
        self._release(("qkv_w", "qkv_b"))

    def release_mlp(self):
        self._release(("fc1_w", "fc2_w", "fc1_b", "fc2_b"))

    def _release(self, names):
        self._shapes = getattr(self, "_shapes", {})
        for n, t in self._fused_tensors():
            if n in names and t.numel():
                self._shapes[n] = tuple(t.shape)
                t.data = torch.empty(0, dtype=t.dtype, device=t.device)

    def release_memory(self):
        """Drop the fused layer's matrices (the client's copies stay); `reset_params` brings them back."""
        self.release_qkv()
        self._release(("o_w", "o_b"))
        self.release_mlp()
        self._released = True

    def reset_qkv(self):
        self._reset(("qkv_w", "qkv_b"))

    def reset_mlp(self):
        self._reset(("fc1_w", "fc2_w", "fc1_b", "fc2_b"))

    def _reset(self, names):
        for n, t in self._fused_tensors():
            if n in names and n in getattr(self, "_shapes", {}) and not t.numel():
                t.data = torch.empty(self._shapes[n], dtype=t.dtype, device=t.device)

    def reset_params(self):
        self._reset(("qkv_w", "qkv_b", "o_w", "o_b", "fc1_w", "fc2_w", "fc1_b", "fc2_b"))
        self._released = False
        super().initialize_tensors()
        if hasattr(self, "transpose"):
            self.transpose()
        self.copy_data_to_new_module()

    def set_params_wo_copy(self, Z3_enabled=False):
        """Point the fused layer at the client's own storage where the layouts agree (unsharded [out, in] weights
        of the same dtype on the same device): the attention output and the second MLP matrix. Fused QKV and the
        first MLP matrix are concatenations, so they are copied."""
        self.set_attn_params_wo_copy(Z3_enabled=Z3_enabled)
        self.set_mlp_params_wo_copy(Z3_enabled=Z3_enabled)

    def _alias(self, name, src):
        dst = getattr(self.module.layer, name, None)
        if dst is None or src is None:
            return False
        if self.mp_size > 1 or src.dtype != dst.dtype or src.device != dst.device or \
                tuple(src.shape) != tuple(dst.shape) or not src.is_contiguous():
            with torch.no_grad():
                dst.copy_(src.reshape(dst.shape)) if src.numel() == dst.numel() else None
            return False
        dst.data = src.data
        return True

    def set_attn_params_wo_copy(self, **kwargs):
        self._alias("o_w", self._dense_w)
        self._alias("o_b", self._dense_b)

    def set_mlp_params_wo_copy(self, **kwargs):
        self._alias("fc2_w", self._out_w)
        self._alias("fc2_b", self._out_b)


class HybridMegatronContainer(MegatronContainer, HybridEngineContainer):
    """Megatron layer in the hybrid engine: the v2 QKV re-layout is redone at every switch to inference
    (`transform_for_inference` calls `transpose`); training keeps the checkpoint's own layout."""

    def _align_qkv(self, x):
        return self._align_qkv_transposed(x)

    def _partition_qkv(self, x):
        """Inverse of `_align_qkv`: [q | k | v] blocks back to per-head [heads, 3, head_dim] rows."""
        if x is None:
            return None
        heads = self.num_attention_heads
        hd = x.shape[0] // (3 * heads)
        return x.view(3, heads, hd, *x.shape[1:]).transpose(0, 1).reshape(x.shape)


class HybridSplitQKVContainer(HybridEngineContainer):
    """Clients with separate q / k / v projections: the policy's `attention()` concatenates them, and this mixin
    keeps the three parts addressable (for LoRA on a single projection, or partial refreshes)."""

    def set_q_k_v(self):
        """Set `self.qw, self.qb, self.kw, self.kb, self.vw, self.vb` from the client layer."""
        raise NotImplementedError("a split-QKV container names its three projections in set_q_k_v()")

    def set_attention(self, qkvw, qkvb, dense_w, dense_b):
        self._qkvw, self._qkvb, self._dense_w, self._dense_b = qkvw, qkvb, dense_w, dense_b
        self.set_q_k_v()

    def get_attn_params(self):
        return [self.qw, self.qb, self.kw, self.kb, self.vw, self.vb, self._dense_w, self._dense_b]

    def attention_qkv_mp(self, mp_replace=None, reversed_dim=False):
        """Fused [q | k | v] from the three parts (tensor-parallel slicing happens in `copy_data_to_new_module`)."""
        self.set_q_k_v()
        self._qkvw = torch.cat([self.qw, self.kw, self.vw], 0)
        self._qkvb = None if self.qb is None else torch.cat([self.qb, self.kb, self.vb], 0)
        return self._qkvw, self._qkvb

    def reset_qkv(self):
        super().reset_qkv()
        if self.module is not None and self.mp_size == 1:
            qkvw, qkvb = self.attention_qkv_mp()
            with torch.no_grad():
                self.module.layer.qkv_w.copy_(qkvw.reshape(self.module.layer.qkv_w.shape))
                if qkvb is not None and getattr(self.module.layer, "qkv_b", None) is not None:
                    self.module.layer.qkv_b.copy_(qkvb.reshape(self.module.layer.qkv_b.shape))


class HybridGatedMLPContainer(HybridEngineContainer):
    """Clients with separate gate / up projections: fused as [gate | up] rows for the gated-activation kernel."""

    def set_mlp_gate(self):
        """Set `self.inter_up_w, self.inter_up_b, self.inter_gate_w, self.inter_gate_b` from the client layer."""
        raise NotImplementedError("a gated-MLP container names its two projections in set_mlp_gate()")

    def set_mlp(self, _h4h_w, _h4h_b, _4hh_w, _4hh_b):
        self._inter_w, self._inter_b, self._out_w, self._out_b = _h4h_w, _h4h_b, _4hh_w, _4hh_b
        self.set_mlp_gate()

    def get_mlp_params(self):
        return [self.inter_up_w, self.inter_up_b, self.inter_gate_w, self.inter_gate_b, self._out_w, self._out_b]

    def mlp_inter_mp(self, mp_replace=None, reversed_dim=False):
        self.set_mlp_gate()
        self._inter_w = torch.cat([self.inter_gate_w, self.inter_up_w], 0)
        self._inter_b = None if self.inter_up_b is None else torch.cat([self.inter_gate_b, self.inter_up_b], 0)
        return self._inter_w, self._inter_b
