"""Compression schedule (reference `compression/scheduler.py`): each technique switches on when the training step
reaches its `schedule_offset`; after that
  * sparse pruning with `schedule_offset_end` anneals the dense ratio from 1.0 to the target between the offset and
    the end (cubic, as gradual magnitude pruning does), refreshing masks every `schedule_offset_stride` steps —
    method `snip_momentum` scores weights by |w * grad| with a momentum-averaged score;
  * weight quantization with `quantize_weight_in_forward = false` quantises the weights in place after every
    optimizer step (the reference rewrites `optimizer.step` for the same effect); masks of the other pruning
    techniques are refreshed on the same cadence."""
import torch

from .basic_layer import fake_quant
from .config import TECHNIQUES
from .helper import recursive_getattr


def _enable(m, tech, shared, params):
    if tech == "weight_quantization" and hasattr(m, "enable_weight_quantization"):
        m.enable_weight_quantization(params["start_bits"], params["target_bits"], params["quantization_period"],
                                     shared["quantize_weight_in_forward"], shared["quantization_type"],
                                     shared["quantize_groups"])
    elif tech == "activation_quantization" and hasattr(m, "enable_activation_quantization"):
        m.enable_activation_quantization(params["bits"], shared["quantization_type"], shared["range_calibration"])
    elif tech == "sparse_pruning" and hasattr(m, "enable_sparse_pruning"):
        start_ratio = 1.0 if shared.get("schedule_offset_end") else params["dense_ratio"]
        m.enable_sparse_pruning(start_ratio, "topk" if shared["method"] == "topk" else "l1")
    elif tech == "row_pruning" and hasattr(m, "enable_row_pruning"):
        m.enable_row_pruning(params["dense_ratio"], shared["method"])
    elif tech == "head_pruning" and hasattr(m, "enable_head_pruning"):
        m.enable_head_pruning(params["dense_ratio"], shared["method"], shared["num_heads"])
    elif tech == "channel_pruning" and hasattr(m, "enable_channel_pruning"):
        m.enable_channel_pruning(params["dense_ratio"], shared["method"])
    else:
        return False
    return True


class compression_scheduler:

    def __init__(self, model, compression_config):
        from .config import get_compression_config
        self.model = model
        self.cc = get_compression_config(compression_config)
        self.enabled = set()
        self._step = 0
        self._snip = {}
        self.moq_external = False  # the engine's MoQ quantizer (runtime/quantize.py) owns the in-place weight quant

    @property
    def weight_quantization_enabled(self):
        return any(t == "weight_quantization" for (t, _) in self.enabled)

    def _plan(self):
        return getattr(self.model, "_ds_compression_plan", [])

    @torch.no_grad()
    def _gradual_sparse(self, m, shared, params, step):
        lo, hi = shared["schedule_offset"], shared["schedule_offset_end"]
        stride = max(int(shared.get("schedule_offset_stride") or 1), 1)
        if step > hi or (step - lo) % stride:
            return
        frac = min(max((step - lo) / max(hi - lo, 1), 0.0), 1.0)
        target = float(params["dense_ratio"])
        m.sparse_pruning_ratio = target + (1.0 - target) * (1.0 - frac)**3
        if shared["method"] == "snip_momentum" and m.weight.grad is not None:
            sc = (m.weight.detach() * m.weight.grad.detach()).abs().float()
            prev = self._snip.get(id(m))
            self._snip[id(m)] = sc if prev is None else 0.9 * prev + 0.1 * sc
            from .basic_layer import _topk_mask
            m.sparse_pruning_mask.copy_(_topk_mask(self._snip[id(m)], m.sparse_pruning_ratio))
        else:
            m.update_masks()

    def _check(self, techs, step):
        """Switch on / advance the given techniques at training step `step`."""
        for (tech, n, shared, params, related) in self._plan():
            if tech not in techs:
                continue
            m = recursive_getattr(self.model, n)
            key = (tech, n)
            if key not in self.enabled:
                if step < shared.get("schedule_offset", 0):
                    continue
                if _enable(m, tech, shared, params) and hasattr(m, "update_masks"):
                    m.update_masks()
                self.enabled.add(key)
                continue
            if tech == "sparse_pruning" and shared.get("schedule_offset_end") and getattr(m, "sparse_pruning_enabled",
                                                                                          False):
                self._gradual_sparse(m, shared, params, step)
            elif tech == "weight_quantization" and not shared["quantize_weight_in_forward"] and \
                    getattr(m, "weight_quantization_enabled", False) and not self.moq_external:
                bits = getattr(m, "wq_bits", getattr(m, "wq_target_bits", 8))
                with torch.no_grad():
                    m.weight.copy_(fake_quant(m.weight, bits, m.wq_groups, m.wq_symmetric))

    def step(self, step_zero_check=None):
        step = self._step if step_zero_check is None else int(step_zero_check)
        self._check(TECHNIQUES, step)
        self._step = step + 1

    # ---- the reference's per-technique entry points (`compression/scheduler.py:66-160`)
    @property
    def training_steps(self):
        return self._step

    @training_steps.setter
    def training_steps(self, v):
        self._step = int(v)

    def make_init(self):
        """{technique: {"enabled", "shared_parameters", "different_groups": [[group, [module names], params]]}} —
        the plan `init_compression` attached to the model, regrouped per technique."""
        out = {}
        for tech in TECHNIQUES:
            shared = self.cc[tech]["shared_parameters"]
            groups = {}
            for (t, n, _, params, _) in self._plan():
                if t == tech:
                    groups.setdefault(id(params), [None, [], params])[1].append(n)
            names = list(self.cc[tech]["different_groups"])
            rows = list(groups.values())
            for i, row in enumerate(rows):
                row[0] = names[i] if i < len(names) else f"group_{i}"
            out[tech] = {"enabled": shared["enabled"], "shared_parameters": shared, "different_groups": rows}
        self.different_compression_methods = out
        return out

    def check_weight_quantization(self):
        self._check(("weight_quantization", ), self._step)

    def check_activation_quantization(self):
        self._check(("activation_quantization", ), self._step)

    def check_sparse_pruning(self):
        self._check(("sparse_pruning", ), self._step)

    def check_head_pruning(self):
        self._check(("head_pruning", ), self._step)

    def check_row_pruning(self):
        self._check(("row_pruning", ), self._step)

    def check_channel_pruning(self):
        self._check(("channel_pruning", ), self._step)

    def check_all_modules(self):
        self._check(TECHNIQUES, self._step)
