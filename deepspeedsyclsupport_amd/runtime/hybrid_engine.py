"""Hybrid engine for RLHF (reference `runtime/hybrid_engine.py:32-446`): one engine that trains (ZeRO, any stage)
and generates (kernel-injected inference) with the SAME weights.

generate():
  1. fuse LoRA adapters into the base weights (modules exposing fuse_lora_weight / unfuse_lora_weight, the
     DeepSpeed-Chat convention);
  2. make the persistent `DSInferenceModel` (paged KV cache, HIP decode kernels, optional HIP-graph decode) hold the
     current weights:
       * ZeRO-0/1/2 with inference_tp_size 1: it SHARES the training tensors — every inference weight is an alias of
         the module's parameter (q/k/v and gate/up stay separate tensors applied side by side), so the optimizer's
         in-place updates and LoRA fusing are visible without any copy and no second weight set exists;
       * ZeRO-3 and/or inference_tp_size > 1 (reference `hybrid_engine.py:115,183-230,316-337`): a TP-sharded
         inference model (1/tp of the weights per rank) refilled ONE LAYER AT A TIME — gather that layer's partitions,
         copy this rank's shard, release — and only when the weights changed (optimizer step / LoRA) since the last
         refresh;
  3. with inference_tp_size > 1 the ranks of a TP group pool their prompts, generate together on the sharded model
     (RCCL all-reduce per block) and each keeps its own rows;
  4. unfuse LoRA (and, with release_inference_cache, drop the KV cache).
Models without an injection policy fall back to the module's own `generate` under fully gathered parameters.
"""
import time

import torch

from .. import comm as dist
from ..utils.logging import log_dist
from .engine import DeepSpeedEngine


class DeepSpeedHybridEngine(DeepSpeedEngine):
    inference_mp_group = None

    def __init__(self, args, model, **kwargs):
        super().__init__(args, model, **kwargs)
        self.hcfg = self._config.hybrid_engine
        self._inference = None        # InferenceEngine over the injected model
        self._ds_model = None
        self._extract = None
        self._generate_calls = 0
        self._t_generate = 0.0
        self._t_last = 0.0
        self.is_lora_fused = False
        self._in_generate = False

    # ------------------------------------------------------------------------------------------ helpers
    def _lora_modules(self):
        return [m for m in self.module.modules() if hasattr(m, "fuse_lora_weight") and hasattr(m, "unfuse_lora_weight")]

    def fuse_lora_weight(self):
        for m in self._lora_modules():
            m.fuse_lora_weight()
        self.is_lora_fused = True

    def unfuse_lora_weight(self):
        for m in self._lora_modules():
            m.unfuse_lora_weight()
        self.is_lora_fused = False

    def _gathered(self, params=None):
        if self.zero_optimization_partition_weights():
            from .zero.partition_parameters import GatheredParameters
            return GatheredParameters(list(self.module.parameters()) if params is None else list(params))
        return _Null()

    def _tp(self):
        """(group, size, rank) of this rank's inference TP group: consecutive ranks, created collectively once."""
        if not hasattr(self, "_tp_info"):
            tp = max(int(self.hcfg.inference_tp_size), 1)
            world, rank = dist.get_world_size(), dist.get_rank()
            if tp == 1 or world == 1:
                self._tp_info = (None, 1, 0)
            else:
                if world % tp:
                    raise ValueError(f"inference_tp_size {tp} must divide the world size {world}")
                mine = None
                for g in range(world // tp):
                    grp = dist.new_group(list(range(g * tp, (g + 1) * tp)))
                    if g == rank // tp:
                        mine = grp
                self._tp_info = (mine, tp, rank % tp)
        return self._tp_info

    def _layer_container(self, num_layers):
        """The ModuleList holding the decoder layers (per-layer gathers under ZeRO-3)."""
        for _, m in self.module.named_modules():
            if isinstance(m, torch.nn.ModuleList) and len(m) == num_layers:
                return m
        return None

    def _weights_version(self):
        return (getattr(self, "global_steps", 0), self.is_lora_fused, id(self))

    def _share_into(self, ds, spec, top, layers):
        """Alias the inference model's weights to the training tensors (ZeRO-0/1/2, TP 1): no copy. The model was
        built on the meta device, so each parameter is REPLACED by one wrapping the training tensor's storage."""
        dev = self.device

        def put(mod, name, t):
            if getattr(mod, name, None) is None or t is None:
                return
            mod._parameters[name] = torch.nn.Parameter(t, requires_grad=False)

        def alias(mod, name, src):
            p = getattr(mod, name, None)
            if p is None or src is None:
                return
            src = src.detach()
            if src.dtype != p.dtype or src.shape != p.shape:  # (rare) dtype / shape mismatch: own copy
                src = src.to(dtype=p.dtype, device=dev).reshape(p.shape).clone()
            put(mod, name, src)

        for layer, lw in zip(ds.layers, layers):
            layer.split_w["qkv_w"] = [lw["q_w"].detach(), lw["k_w"].detach(), lw["v_w"].detach()]
            if lw.get("q_b") is not None:
                layer.split_b["qkv_w"] = [lw["q_b"], lw["k_b"], lw["v_b"]]
            fused_mlp = "gate_w" in lw
            if fused_mlp:
                layer.split_w["fc1_w"] = [lw["gate_w"].detach(), lw["up_w"].detach()]
                if lw.get("gate_b") is not None:
                    layer.split_b["fc1_w"] = [lw["gate_b"], lw["up_b"]]
            else:
                alias(layer, "fc1_w", lw["fc1_w"])
                alias(layer, "fc1_b", lw.get("fc1_b"))
            for name in ("qkv_w", "qkv_b") + (("fc1_w", "fc1_b") if fused_mlp else ()):
                p = getattr(layer, name, None)
                if p is not None:
                    put(layer, name, torch.empty(0, dtype=p.dtype, device=dev))
            alias(layer, "o_w", lw["o_w"])
            alias(layer, "o_b", lw.get("o_b"))
            alias(layer, "fc2_w", lw["fc2_w"])
            alias(layer, "fc2_b", lw.get("fc2_b"))
            for n in ("ln1_w", "ln1_b", "ln2_w", "ln2_b"):
                alias(layer, n, lw.get(n))
            if spec.shared_parallel_norm:
                alias(layer, "ln2_w", lw["ln1_w"])
                alias(layer, "ln2_b", lw.get("ln1_b"))
        alias(ds, "embed", top["embed"])
        if spec.embed_norm:
            alias(ds, "embed_ln_w", top["embed_ln_w"])
            alias(ds, "embed_ln_b", top["embed_ln_b"])
        alias(ds, "norm_w", top["norm_w"])
        alias(ds, "norm_b", top.get("norm_b"))
        if ds.lm_head.shape[0] == top["lm_head"].shape[0]:
            alias(ds, "lm_head", top["lm_head"])
            alias(ds, "lm_head_b", top.get("lm_head_b"))
        else:  # vocab padding: keep an own padded copy
            lm = torch.zeros(ds.lm_head.shape, dtype=ds.dtype, device=dev)
            lm[:top["lm_head"].shape[0]].copy_(top["lm_head"].detach())
            put(ds, "lm_head", lm)
        if ds.pos_embed is not None:
            pe = top["pos_embed"].detach()
            t = torch.zeros(ds.pos_embed.shape, dtype=ds.dtype, device=dev)
            n = min(pe.shape[0], t.shape[0])
            t[:n].copy_(pe[:n])
            put(ds, "pos_embed", t)
        self._materialize(ds)

    def _materialize(self, ds):
        """Give every parameter still on the meta device real (zero) storage and rebuild the position tables."""
        from ..inference.model_implementations.transformer import alibi_slopes
        from ..ops import reference
        for mod in ds.modules():
            for name, p in list(mod._parameters.items()):
                if p is not None and p.device.type == "meta":
                    mod._parameters[name] = torch.nn.Parameter(
                        torch.zeros(p.shape, dtype=p.dtype, device=self.device), requires_grad=False)
        spec = ds.spec
        if ds.rope_cos is not None and ds.rope_cos.device.type == "meta":
            cos, sin = reference.rope_tables(max(spec.max_positions, 2048) * 2, spec.rotary_dim, spec.rope_theta,
                                             device=self.device)
            ds.rope_cos, ds.rope_sin = cos, sin
        if ds.alibi is not None and ds.alibi.device.type == "meta":
            hq = spec.num_heads // ds.tp_size
            ds.alibi = alibi_slopes(spec.num_heads)[ds.tp_rank * hq:(ds.tp_rank + 1) * hq].contiguous().to(self.device)
        ds.device = self.device

    def _copy_into(self, ds, spec):
        """TP-sharded copy, one decoder layer gathered at a time (ZeRO-3 partitions are never gathered at once)."""
        from ..inference.model_implementations import convert
        container = self._layer_container(spec.num_layers)
        r, tp = ds.tp_rank, ds.tp_size
        for i, layer in enumerate(ds.layers):
            params = container[i].parameters() if container is not None else self.module.parameters()
            with self._gathered(params):
                _, _, layers = convert.extract(self.module)
                with torch.no_grad():
                    for name, t in convert.shard_layer(spec, layers[i], r, tp).items():
                        p = getattr(layer, name)
                        if p is not None and t is not None:
                            p.data.copy_(t.detach().to(p.dtype))
        per_layer = set(id(p) for p in container.parameters()) if container is not None else set()
        rest = [p for p in self.module.parameters() if id(p) not in per_layer]
        with self._gathered(rest):
            _, top, _ = convert.extract(self.module)
            with torch.no_grad():
                convert.load_into(ds, top, [])

    def _refresh_inference_model(self):
        from ..inference.config import DeepSpeedInferenceConfig
        from ..inference.engine import InferenceEngine
        from ..inference.model_implementations import convert
        if not convert.supported(self.module):
            return None
        group, tp, r = self._tp()
        zero3 = self.zero_optimization_partition_weights()
        share = not zero3 and tp == 1
        dtype = self._dtype() if self._dtype() in (torch.bfloat16, torch.float16) else torch.float32
        if self._ds_model is None:
            from ..inference.model_implementations.transformer import DSInferenceModel
            spec, top, layers = convert.extract(self.module)
            spec.max_positions = max(spec.max_positions, self.hcfg.max_out_tokens)
            # shared weights: build on the meta device so no second weight set is ever allocated
            self._ds_model = DSInferenceModel(spec, group, tp, r, dtype,
                                              torch.device("meta") if share else self.device)
            self._loaded_version = None
            if share:
                self._share_into(self._ds_model, spec, top, layers)
                self._loaded_version = "shared"
            cfg = DeepSpeedInferenceConfig(dtype=dtype, max_tokens=self.hcfg.max_out_tokens)
            self._inference = InferenceEngine.from_ds_model(self._ds_model, cfg, tp_group=group, tp_size=tp,
                                                            tp_rank=r)
        if self._loaded_version != "shared" and self._loaded_version != self._weights_version():
            self._copy_into(self._ds_model, self._ds_model.spec)
            self._loaded_version = self._weights_version()
        return self._inference

    def _tp_generate(self, inf, input_ids, **kwargs):
        """inference_tp_size > 1: pool the TP group's prompts, generate once on the sharded model, keep own rows."""
        group, tp, r = self._tp()
        if tp == 1:
            return inf.generate(input_ids, **kwargs)
        parts = [torch.empty_like(input_ids) for _ in range(tp)]
        dist.all_gather(parts, input_ids.contiguous(), group=group)
        out = inf.generate(torch.cat(parts, 0), **kwargs)
        B = input_ids.shape[0]
        return out[r * B:(r + 1) * B]

    # ------------------------------------------------------------------------------------------ API
    @torch.no_grad()
    def generate(self, *inputs, **kwargs):
        t0 = time.time()
        self._in_generate = True
        was_training = self.module.training
        self.module.eval()
        try:
            if self._lora_modules():
                with self._gathered():
                    self.fuse_lora_weight()
            try:
                inf = self._refresh_inference_model()
                if inf is not None:
                    ids = inputs[0] if inputs else kwargs.pop("input_ids")
                    out = self._tp_generate(inf, ids.to(self.device), **kwargs)
                else:
                    with self._gathered():
                        out = self.module.generate(*inputs, **kwargs)
            finally:
                if self.is_lora_fused:
                    with self._gathered():
                        self.unfuse_lora_weight()
        finally:
            self._in_generate = False
            if was_training:
                self.module.train()
            if self.hcfg.release_inference_cache and self._ds_model is not None:
                self._ds_model.cache = None
                if self._inference is not None:
                    self._inference._graphs.clear()
        self._generate_calls += 1
        self._t_last = time.time() - t0
        self._t_generate += self._t_last
        return out

    # ------------------------------------------------------------------------------------------ per-layer containers
    # Architectures without a whole-model converter can still run their transformer layers fused: every client
    # layer a policy of `module_inject.containers.replace_policies` matches gets a hybrid container (reference
    # `runtime/hybrid_engine.py:84-160, 280-330`), and `fused_layers()` swaps the layers' forwards for the fused
    # ones while it is open.
    def populate_all_inference_policies(self):
        from ..module_inject.containers import replace_policies
        self.inference_policies = {}
        for pol in replace_policies:
            try:
                pol(None)            # policies resolve their client layer class on first construction
            except Exception:
                pass
            classes = pol._orig_layer_class
            for c in (classes if isinstance(classes, (list, tuple)) else [classes]):
                if c is not None:
                    self.inference_policies[c] = pol
        return self.inference_policies

    def new_inference_container(self, orig_layer, policy_cls, layer_id):
        from ..inference.config import DeepSpeedInferenceConfig
        from ..module_inject import containers as C
        from ..module_inject.container_features import HybridEngineContainer
        policy = policy_cls(orig_layer, inference=True)
        dtype = self._dtype() if self._dtype() in (torch.bfloat16, torch.float16) else torch.float32
        base = C.BaseTransformerContainer
        for cls in type(policy).__mro__:
            if cls in C._CONTAINERS:
                base = C._CONTAINERS[cls]
                break
        kind = type("Hybrid" + base.__name__, (HybridEngineContainer, base), {})
        cfg = DeepSpeedInferenceConfig(dtype=dtype, max_out_tokens=self.hcfg.max_out_tokens)
        cont = kind(policy=policy, config=cfg, model_config=getattr(self.module, "config", None), layer_id=layer_id,
                    child=orig_layer)
        cont.create_ds_model_config()
        cont.create_module()
        return cont

    def create_inference_containers(self, module=None, layer_id=0):
        module = self.module if module is None else module
        for child in module.children():
            pol = self.inference_policies.get(type(child))
            if pol is not None:
                self._inference_containers.append(self.new_inference_container(child, pol, layer_id))
                self._orig_modules.append(child)
                self._orig_fwds.append(child.forward)
                layer_id += 1
            else:
                layer_id = self.create_inference_containers(child, layer_id)
        return layer_id

    def create_inference_module(self):
        self._inference_containers, self._orig_modules, self._orig_fwds = [], [], []
        self.populate_all_inference_policies()
        self.create_inference_containers(self.module)
        self.lora_params = [c.get_lora_params() for c in self._inference_containers]
        return len(self._inference_containers)

    def fused_layers(self):
        """Context manager: refresh every layer container from the (just trained) client weights and run the
        client layers through their fused counterparts until it closes."""
        import contextlib
        from ..module_inject.containers import _InjectedLayer

        @contextlib.contextmanager
        def ctx():
            if not getattr(self, "_inference_containers", None):
                self.create_inference_module()
            with self._gathered():
                for c in self._inference_containers:
                    c.transform_for_inference()
            try:
                for c, m in zip(self._inference_containers, self._orig_modules):
                    m.forward = _InjectedLayer(c.module, c.policy.return_tuple).forward
                yield self._inference_containers
            finally:
                for m, f in zip(self._orig_modules, self._orig_fwds):
                    m.forward = f
                if self.hcfg.release_inference_cache:
                    for c in self._inference_containers:
                        c.release_memory()

        return ctx()

    def retake_inference_cache(self):
        """Bring back what `release_inference_cache` dropped (the KV cache of the whole-model path is re-allocated
        by the next generate on its own)."""
        for c in getattr(self, "_inference_containers", []):
            if c._released:
                c.reset_params()

    def unfuse_lora_weight_non_pinned(self):
        with self._gathered():
            self.unfuse_lora_weight()

    def convert_to_linear_transposed(self, model):
        """The reference re-wraps nn.Linear to hold transposed weights for its GEMMs; the GEMMs here take the
        [out, in] weights as stored, so there is nothing to convert."""
        return model

    def eval(self):
        self.module.eval()
        return self

    def train(self, mode=True):
        self.module.train(mode)
        return self

    def generate_latency(self):
        return self._t_last, self._t_generate / max(self._generate_calls, 1)

    def print_generate_stats(self):
        last, avg = self.generate_latency()
        log_dist(f"hybrid engine: generate calls={self._generate_calls} last={last * 1e3:.1f} ms "
                 f"avg={avg * 1e3:.1f} ms", ranks=[0])


class _Null:

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
