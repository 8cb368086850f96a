"""Build a model whose eligible weights are quantised as they are created (reference
`inference/quantization/quantization_context.py`: a ZeRO-3 `Init` context that also quantises).

    with QuantizationContext(config_dict_or_path=ds_config):
        model = AutoModelForCausalLM.from_config(cfg)

On exit the modules constructed inside are passed through the post-init group-wise quantiser
(`quantization._init_group_wise_weight_quantization`) with the `weight_quantization.quantized_initialization`
settings of the config; with ZeRO stage 3 in the config the construction also runs under `zero.Init`, so the full
weights never exist on one device."""
import contextlib

import torch.nn as nn

from .quantization import _init_group_wise_weight_quantization


class QuantizationContext(contextlib.AbstractContextManager):

    def __init__(self, config_dict_or_path, param_swapper=None):
        import json
        cfg = config_dict_or_path
        if isinstance(cfg, str):
            with open(cfg) as f:
                cfg = json.load(f)
        self.ds_config = cfg
        self._zero = None
        self._made = []

    def __enter__(self):
        if self.ds_config.get("zero_optimization", {}).get("stage", 0) == 3:
            from ...runtime.zero.partition_parameters import Init
            self._zero = Init(config_dict_or_path=self.ds_config)
            self._zero.__enter__()
        made = self._made
        self._orig_init = orig = nn.Module.__init__

        def tracking_init(module, *a, **k):
            orig(module, *a, **k)
            made.append(module)

        nn.Module.__init__ = tracking_init
        return self

    def __exit__(self, *exc):
        nn.Module.__init__ = self._orig_init
        if self._zero is not None:
            self._zero.__exit__(*exc)
        if exc[0] is None:
            inner = {id(c) for m in self._made for c in m.children()}
            for root in [m for m in self._made if id(m) not in inner]:
                _init_group_wise_weight_quantization(root, self.ds_config)
        self._made.clear()
        return False
