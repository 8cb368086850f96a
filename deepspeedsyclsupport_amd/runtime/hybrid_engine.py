"""Hybrid engine for RLHF (reference `runtime/hybrid_engine.py:32-446`): one engine that trains (ZeRO, any stage)
and generates (kernel-injected inference) with the SAME weights.

generate():
  1. (ZeRO-3) gather the partitioned parameters once for the whole rollout;
  2. fuse LoRA adapters into the base weights (modules exposing fuse_lora_weight / unfuse_lora_weight, the
     DeepSpeed-Chat convention);
  3. refresh a persistent `DSInferenceModel` built from the training module (paged KV cache, HIP decode kernels,
     optional HIP-graph decode) — refresh is a device-to-device weight copy, no re-conversion;
  4. generate, then unfuse LoRA and release the gathered parameters (and, with release_inference_cache, the cache).
Models without an injection policy fall back to the module's own `generate` under the gathered parameters.
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

    def _gathered(self):
        if self.zero_optimization_partition_weights():
            from .zero.partition_parameters import GatheredParameters
            return GatheredParameters(list(self.module.parameters()))
        return _Null()

    def _refresh_inference_model(self):
        from ..inference.config import DeepSpeedInferenceConfig
        from ..inference.engine import InferenceEngine
        from ..inference.model_implementations import convert
        if not convert.supported(self.module):
            return None
        spec, top, layers = convert.extract(self.module)
        dtype = self._dtype() if self._dtype() in (torch.bfloat16, torch.float16) else torch.float32
        if self._ds_model is None:
            from ..inference.model_implementations.transformer import DSInferenceModel
            spec.max_positions = max(spec.max_positions, self.hcfg.max_out_tokens)
            self._ds_model = DSInferenceModel(spec, None, 1, 0, dtype, self.device)
            cfg = DeepSpeedInferenceConfig(dtype=dtype, max_tokens=self.hcfg.max_out_tokens)
            self._inference = InferenceEngine.from_ds_model(self._ds_model, cfg)
        with torch.no_grad():
            convert.load_into(self._ds_model, top, layers)
        return self._inference

    # ------------------------------------------------------------------------------------------ API
    @torch.no_grad()
    def generate(self, *inputs, **kwargs):
        t0 = time.time()
        self._in_generate = True
        was_training = self.module.training
        self.module.eval()
        try:
            with self._gathered():
                if self._lora_modules():
                    self.fuse_lora_weight()
                try:
                    inf = self._refresh_inference_model()
                    if inf is not None:
                        out = inf.generate(*inputs, **kwargs)
                    else:
                        out = self.module.generate(*inputs, **kwargs)
                finally:
                    if self.is_lora_fused:
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
