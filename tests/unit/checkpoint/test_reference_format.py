"""Loading reference-layout ZeRO checkpoints.

No checkpoint produced by the reference ships in `/root/reference`, so these tests synthesise shard files exactly as
the reference's save code lays them out — ZeRO-1/2: `stage_1_and_2.py:2102-2146` (`single_partition_of_fp32_groups`
per optimizer group = the rank's slice of the group's flat tensor, flattened in `param_shapes` order and padded to a
multiple of 2*dp; `base_optimizer_state` = the torch optimizer state of those flat partitions; a pickled
`LossScaler` object), ZeRO-3: `stage3.py:2382-2395` (`fp32_flat_groups`, every parameter cut into
ceil(numel / dp) pieces) — and check that the engine restores every fp32 master and Adam moment from them at the
same and at a different data-parallel size. Byte parity with real reference files remains unpinned.
"""
import math
import os
from collections import OrderedDict

import pytest
import torch

from deepspeedsyclsupport_amd.checkpoint import zero_checkpoint as zc

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama


def _ref_values(seed=0):
    model = tiny_llama(seed=seed)
    g = torch.Generator().manual_seed(123)
    vals = OrderedDict()
    for n, p in model.named_parameters():
        vals[n] = (p.detach().float().clone(), torch.randn(p.shape, generator=g) * 1e-3,
                   torch.rand(p.shape, generator=g) * 1e-6)
    return vals


def _loss_scaler_obj():
    stubs = zc._reference_pickle_stubs()
    cls = [c for c in stubs if c.__name__ == "LossScaler"][0]
    obj = cls.__new__(cls)
    obj.__dict__.update({"cur_scale": 1.0, "dynamic": False})
    return obj


class _fake_reference_modules:
    """Make the stub classes importable under the reference's module paths while the synthetic files are pickled
    (the pickler checks importability); removed afterwards."""

    def __enter__(self):
        import sys
        import types
        self.added = []
        for cls in zc._reference_pickle_stubs():
            parts = cls.__module__.split(".")
            for i in range(1, len(parts) + 1):
                name = ".".join(parts[:i])
                if name not in sys.modules:
                    sys.modules[name] = types.ModuleType(name)
                    self.added.append(name)
            setattr(sys.modules[cls.__module__], cls.__qualname__, cls)
        return self

    def __exit__(self, *a):
        import sys
        for name in self.added:
            sys.modules.pop(name, None)


def write_reference_zero2(d, vals, world, step=3):
    with _fake_reference_modules():
        _write_reference_zero2(d, vals, world, step)


def write_reference_zero3(d, vals, world, step=3):
    with _fake_reference_modules():
        _write_reference_zero3(d, vals, world, step)


def _write_reference_zero2(d, vals, world, step=3):
    os.makedirs(d, exist_ok=True)
    names = list(vals.keys())
    shapes = OrderedDict((n, vals[n][0].shape) for n in names)
    torch.save({"module": {n: vals[n][0].bfloat16() for n in names}, "param_shapes": [shapes],
                "global_steps": step, "dp_world_size": world}, os.path.join(d, "mp_rank_00_model_states.pt"))
    flats = [torch.cat([vals[n][i].reshape(-1) for n in names]) for i in range(3)]
    align = 2 * world
    pad = (-flats[0].numel()) % align
    flats = [torch.nn.functional.pad(f, (0, pad)) for f in flats]
    P = flats[0].numel() // world
    for r in range(world):
        part = [f[r * P:(r + 1) * P].clone() for f in flats]
        trimmed = part[0][:P - pad] if r == world - 1 else part[0]
        osd = {
            "loss_scaler": _loss_scaler_obj(), "dynamic_loss_scale": False, "overflow": False, "clip_grad": 1.0,
            "base_optimizer_state": {"state": {0: {"step": torch.tensor(float(step)), "exp_avg": part[1],
                                                   "exp_avg_sq": part[2]}},
                                     "param_groups": [{"lr": 1e-2, "betas": (0.9, 0.999), "eps": 1e-8,
                                                       "weight_decay": 0.01, "params": [0]}]},
            "single_partition_of_fp32_groups": [trimmed], "zero_stage": 2, "group_paddings": [pad if r == world - 1
                                                                                               else 0],
            "partition_count": world, "ds_version": "0.12.7", "param_slice_mappings": [OrderedDict()],
        }
        torch.save({"optimizer_state_dict": osd}, os.path.join(d, f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt"))


def _write_reference_zero3(d, vals, world, step=3):
    os.makedirs(d, exist_ok=True)
    names = list(vals.keys())
    shapes = OrderedDict((n, vals[n][0].shape) for n in names)
    for r in range(world):
        pieces = [[], [], []]
        for n in names:
            numel = vals[n][0].numel()
            pn = math.ceil(numel / world)
            for i in range(3):
                flat = torch.nn.functional.pad(vals[n][i].reshape(-1), (0, pn * world - numel))
                pieces[i].append(flat[r * pn:(r + 1) * pn])
        fl = [torch.cat(x) for x in pieces]
        torch.save({"module": {n: torch.empty(0, dtype=torch.bfloat16) for n in names}, "param_shapes": [shapes],
                    "global_steps": step, "dp_world_size": world},
                   os.path.join(d, f"zero_pp_rank_{r}_mp_rank_00_model_states.pt"))
        osd = {"zero_stage": 3, "loss_scaler": _loss_scaler_obj(), "dynamic_loss_scale": False, "overflow": False,
               "partition_count": world,
               "optimizer_state_dict": {"state": {0: {"step": torch.tensor(float(step)), "exp_avg": fl[1],
                                                      "exp_avg_sq": fl[2]}},
                                        "param_groups": [{"lr": 1e-2, "params": [0]}]},
               "fp32_flat_groups": [fl[0]]}
        torch.save({"optimizer_state_dict": osd}, os.path.join(d, f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt"))


@pytest.mark.parametrize("stage", [2, 3])
def test_sources_reconstruct_parameters(stage, tmp_path):
    vals = _ref_values()
    d = str(tmp_path / "t")
    (write_reference_zero2 if stage == 2 else write_reference_zero3)(d, vals, 3)
    src = zc.open_source(d)
    assert isinstance(src, zc.ReferenceZero12Source if stage == 2 else zc.ReferenceZero3Source)
    assert src.step() == 3
    for n, (w, m, v) in vals.items():
        torch.testing.assert_close(src.get(n, "fp32"), w, rtol=0, atol=0)
        torch.testing.assert_close(src.get(n, "exp_avg"), m, rtol=0, atol=0)
        torch.testing.assert_close(src.get(n, "exp_avg_sq"), v, rtol=0, atol=0)


def _load_ref(stage, ckpt, tag, vals_path):
    import sys
    import deepspeedsyclsupport_amd as ds
    assert "deepspeed" not in sys.modules
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    vals = torch.load(vals_path, weights_only=True)
    c = base_config(stage=stage, lr=1e-2, dtype="fp32")
    c["zero_optimization"].update({"reduce_bucket_size": 3000, "stage3_param_persistence_threshold": 100})
    eng, _, _, _ = ds.initialize(model=tiny_llama(seed=9), config=c)
    eng.load_checkpoint(ckpt, tag=tag)
    assert eng.global_steps == 3
    for n, p in eng.module.named_parameters():
        w, m, v = vals[n]
        torch.testing.assert_close(safe_get_full_fp32_param(p), w, rtol=0, atol=0, msg=n)
        torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg"), m, rtol=0, atol=0, msg=n)
        torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg_sq"), v, rtol=0, atol=0, msg=n)
    x = random_tokens(1, 2, 16, seed=4)[0]
    loss = eng(x, labels=x)
    eng.backward(loss)
    eng.step()


@pytest.mark.parametrize("stage", [2, 3])
@pytest.mark.parametrize("world", [2, 1])
def test_engine_loads_reference_layout(stage, world, tmp_path):
    vals = _ref_values()
    vp = str(tmp_path / "vals.pt")
    torch.save(dict(vals), vp)
    ckpt = str(tmp_path / "ck")
    (write_reference_zero2 if stage == 2 else write_reference_zero3)(os.path.join(ckpt, "ref"), vals, 2)
    run_distributed(_load_ref, world, stage, ckpt, "ref", vp)
