"""Parameter types shared by the model containers (reference
`inference/v2/model_implementations/common_parameters/*.py`). `finalize()` returns canonical-dict entries."""
import torch

from .parameter_base import ParameterBase, ParamList, single

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`

EmbeddingParameter = single("embed", "Word embedding table [vocab, hidden].")
UnembedParameter = single("lm_head", "LM head [vocab, hidden].")
InvFreqParameter = single("inv_freq", "Rotary inverse frequencies stored in the checkpoint (recomputed here).")
MoEGatingWeightParameter = single("router_w", "Router [experts, hidden].")


def _keyed(base_doc):

    class _Keyed(ParameterBase):
        """One tensor whose canonical key is chosen by the container (`Cls.as_(key)`)."""
        params: torch.Tensor

        @classmethod
        def as_(cls, key):
            return type(f"{cls.__name__}_{key}", (cls, ), {"key": key, "__annotations__": {}})

    _Keyed.__doc__ = base_doc
    return _Keyed


NormParameter = _keyed("A normalisation gain or bias.")
AttentionOutputParameter = _keyed("Attention output projection weight [hidden, Hq * D] or its bias.")
MLP1Parameter = _keyed("First MLP projection [intermediate, hidden] or its bias (un-gated).")
MLP2Parameter = _keyed("Second MLP projection [hidden, intermediate] or its bias.")
NormParameter.key, AttentionOutputParameter.key = "norm_w", "o_w"
MLP1Parameter.key, MLP2Parameter.key = "fc1_w", "fc2_w"


class UnfusedQKVParameter(ParameterBase):
    """Separate q / k / v projections (weights or biases: `suffix` "w" / "b")."""
    q_params: torch.Tensor
    k_params: torch.Tensor
    v_params: torch.Tensor
    suffix = "w"

    def finalize(self):
        s = self.suffix
        return {f"q_{s}": self.q_params, f"k_{s}": self.k_params, f"v_{s}": self.v_params}


class UnfusedQKVBias(UnfusedQKVParameter):
    suffix = "b"


class FusedQKVParameter(ParameterBase):
    """[q | k | v] stacked along the output dim (equal thirds unless the model has fewer kv heads)."""
    params: torch.Tensor
    suffix = "w"

    def _heads(self):
        spec = self.inference_model.spec
        return spec.num_heads, spec.num_kv_heads, spec.head_dim

    def finalize(self):
        nh, nk, D = self._heads()
        q, k, v = self.params.split([nh * D, nk * D, nk * D], dim=0)
        s = self.suffix
        return {f"q_{s}": q, f"k_{s}": k, f"v_{s}": v}


class FusedQKVBias(FusedQKVParameter):
    suffix = "b"


def megatron_qkv_reshape(param: torch.Tensor, head_size: int, n_heads: int):
    """[heads, (q, k, v), head_size, ...] interleaved rows -> (q, k, v), each [heads * head_size, ...]."""
    rest = param.shape[1:]
    g = param.reshape(n_heads, 3, head_size, *rest)
    return tuple(g[:, i].reshape(n_heads * head_size, *rest) for i in range(3))


class MegatronQKVParameter(FusedQKVParameter):
    """Per-head interleaved fused QKV (BLOOM / GPT-NeoX / Falcon-7B-style without multi-query)."""

    def finalize(self):
        nh, _, D = self._heads()
        q, k, v = megatron_qkv_reshape(self.params, D, nh)
        s = self.suffix
        return {f"q_{s}": q, f"k_{s}": k, f"v_{s}": v}


def transform_gqa_megatron(param: torch.Tensor, head_size: int, n_heads_q: int, n_heads_kv: int):
    """[kv group: (q .. q, k, v), head_size, ...] grouped rows -> (q, k, v)."""
    rest = param.shape[1:]
    g = param.reshape(n_heads_kv, n_heads_q // n_heads_kv + 2, head_size, *rest)
    return (g[:, :-2].reshape(n_heads_q * head_size, *rest), g[:, -2].reshape(n_heads_kv * head_size, *rest),
            g[:, -1].reshape(n_heads_kv * head_size, *rest))


class GQAMegatronQKVParameter(FusedQKVParameter):
    """Grouped fused QKV (Falcon new decoder architecture)."""

    def finalize(self):
        nh, nk, D = self._heads()
        q, k, v = transform_gqa_megatron(self.params, D, nh, nk)
        s = self.suffix
        return {f"q_{s}": q, f"k_{s}": k, f"v_{s}": v}


class GatedMLPParameter(ParameterBase):
    """Gate and up projections of a gated MLP (kept as two canonical entries; the loader stacks this rank's rows of
    each as [gate | up])."""
    gate_params: torch.Tensor
    up_params: torch.Tensor

    def finalize(self):
        return {"gate_w": self.gate_params, "up_w": self.up_params}


class UnfusedMoEGatedMLPParameter(ParameterBase):
    """Per-expert gate (w1) and up (w3) projections -> one [E, 2I, H] tensor, gate rows then up rows."""
    gating_experts: ParamList("n_experts")
    up_experts: ParamList("n_experts")

    def finalize(self):
        return {"experts_gate_up": torch.stack([torch.cat([g, u], dim=0)
                                                for g, u in zip(self.gating_experts, self.up_experts)])}


class UnfusedMoEMLP1Parameter(ParameterBase):
    experts: ParamList("n_experts")

    def finalize(self):
        return {"experts_fc1": torch.stack(list(self.experts))}


class UnfusedMoEMLP2Parameter(ParameterBase):
    experts: ParamList("n_experts")

    def finalize(self):
        return {"experts_down": torch.stack(list(self.experts))}


class FusedMoEGatedMLPParameter(ParameterBase):
    """Experts already stacked in the checkpoint: gate_up [E, 2I, H]."""
    params: torch.Tensor
    key = "experts_gate_up"


class FusedMoEMLP2Parameter(ParameterBase):
    params: torch.Tensor
    key = "experts_down"
