"""Config keys that gate engine behaviour (reference `runtime/engine.py:1219-1265,1475-1500,933-941`,
`runtime/config.py:270-282`): every parsed key either changes what the engine does or is refused loudly."""
import os

import pytest
import torch
import torch.nn as nn

from ..common import run_distributed

H = 16


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(H, H), nn.Tanh(), nn.Linear(H, 4))


def _cfg(**over):
    cfg = {"train_micro_batch_size_per_gpu": 2, "steps_per_print": 1000,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}
    cfg.update(over)
    return cfg


def _steps(eng, n=3, seed=1):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        x, y = torch.randn(2, H, generator=g), torch.randint(0, 4, (2, ), generator=g)
        x = x.to(eng.device)
        loss = nn.functional.cross_entropy(eng(x).float(), y.to(eng.device))
        eng.backward(loss)
        eng.step()
        out.append(float(loss.detach()))
    return out


def _untested(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.runtime.zero.utils import ZeRORuntimeException
    res = {}
    net = _net()
    cfg = _cfg(zero_optimization={"stage": 1})
    del cfg["optimizer"]
    try:
        ds.initialize(model=net, config=cfg, optimizer=torch.optim.RMSprop(net.parameters(), lr=1e-3))
        res["refused"] = False
    except ZeRORuntimeException as e:
        res["refused"] = "zero_allow_untested_optimizer" in str(e)
    net = _net()
    cfg["zero_allow_untested_optimizer"] = True
    eng, *_ = ds.initialize(model=net, config=cfg, optimizer=torch.optim.RMSprop(net.parameters(), lr=1e-3))
    res["losses"] = _steps(eng)
    # offload with an optimizer the host step does not cover is refused at initialize, not at the first step
    net = _net()
    cfg = _cfg(zero_optimization={"stage": 2, "offload_optimizer": {"device": "cpu"}},
               zero_allow_untested_optimizer=True, zero_force_ds_cpu_optimizer=False)
    del cfg["optimizer"]
    try:
        ds.initialize(model=net, config=cfg, optimizer=torch.optim.RMSprop(net.parameters(), lr=1e-3))
        res["offload_refused"] = False
    except ZeRORuntimeException as e:
        res["offload_refused"] = "cannot be offloaded" in str(e)
    # fp16 master weights are refused
    try:
        ds.initialize(model=_net(), config=_cfg(fp16={"enabled": True, "fp16_master_weights_and_grads": True},
                                                zero_optimization={"stage": 2,
                                                                   "offload_optimizer": {"device": "cpu"}}))
        res["fp16_master"] = False
    except NotImplementedError:
        res["fp16_master"] = True
    torch.save(res, out)


def test_untested_optimizer_and_offload_gates(tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_untested, 1, out)
    res = torch.load(out)
    assert res["refused"] and res["offload_refused"] and res["fp16_master"]
    assert all(l == l for l in res["losses"])


def _client_adam_offload(out):
    """A client torch.optim.AdamW under optimizer offload is taken over by the native host Adam and trains like the
    config-built AdamW."""
    import deepspeedsyclsupport_amd as ds
    zo = {"stage": 2, "offload_optimizer": {"device": "cpu"}}
    net = _net()
    cfg = _cfg(zero_optimization=zo)
    del cfg["optimizer"]
    eng, *_ = ds.initialize(model=net, config=cfg,
                            optimizer=torch.optim.AdamW(net.parameters(), lr=1e-2, weight_decay=0.01))
    a = _steps(eng, 4)
    cfg = _cfg(zero_optimization=zo)
    cfg["optimizer"]["params"]["weight_decay"] = 0.01
    eng2, *_ = ds.initialize(model=_net(), config=cfg)
    b = _steps(eng2, 4)
    torch.save({"a": a, "b": b}, out)


def test_client_adamw_with_offload(tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_client_adam_offload, 2, out)
    res = torch.load(out)
    assert res["a"] == pytest.approx(res["b"], rel=1e-5, abs=1e-6)
    assert res["a"][-1] < res["a"][0] + 1.0


def _no_allgather(out, flag):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    eng, *_ = ds.initialize(model=_net(), config=_cfg(zero_optimization={"stage": 2}, disable_allgather=flag,
                                                      dump_state=flag))
    calls = {"ag": 0, "bc": 0}
    ag, bc = dist.all_gather_into_tensor, dist.broadcast

    def count_ag(*a, **k):
        calls["ag"] += 1
        return ag(*a, **k)

    def count_bc(*a, **k):
        calls["bc"] += 1
        return bc(*a, **k)

    dist.all_gather_into_tensor, dist.broadcast = count_ag, count_bc
    losses = _steps(eng, 3)
    dist.all_gather_into_tensor, dist.broadcast = ag, bc
    w = torch.cat([p.detach().float().reshape(-1).cpu() for p in eng.module.parameters()])
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "w": w, "calls": calls}, out)


def test_disable_allgather_broadcasts_instead(tmp_path):
    res = {}
    for flag in (False, True):
        out = str(tmp_path / f"r{int(flag)}.pt")
        run_distributed(_no_allgather, 2, out, flag)
        res[flag] = torch.load(out)
    assert res[True]["calls"]["ag"] == 0 and res[True]["calls"]["bc"] > 0
    assert res[False]["calls"]["ag"] > 0
    assert torch.equal(res[True]["w"], res[False]["w"])
    assert res[True]["losses"] == res[False]["losses"]


def _node_local(save_dir, out):
    """Two 'nodes' of one rank each (LOCAL_RANK 0 on both): with node-local storage both write the model file and the
    `latest` marker into their own folder."""
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    os.environ["LOCAL_RANK"] = "0"
    eng, *_ = ds.initialize(model=_net(), config=_cfg(zero_optimization={"stage": 1},
                                                      checkpoint={"use_node_local_storage": True}))
    _steps(eng, 1)
    mine = os.path.join(save_dir, f"node{dist.get_rank()}")
    eng.save_checkpoint(mine, tag="t")
    ok = os.path.isfile(os.path.join(mine, "latest")) and os.path.isfile(os.path.join(mine, "t",
                                                                                      "mp_rank_00_model_states.pt"))
    got = [None, None]
    dist.all_gather_object(got, ok)
    if dist.get_rank() == 0:
        torch.save(got, out)


def test_node_local_storage_checkpoint(tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_node_local, 2, str(tmp_path), out)
    assert torch.load(out) == [True, True]


def test_fp16_auto_cast_inputs():
    from deepspeedsyclsupport_amd.runtime.engine import DeepSpeedEngine
    x = {"a": torch.randn(2, 3), "b": [torch.arange(3), torch.randn(2, dtype=torch.float64)]}
    y = DeepSpeedEngine._cast_inputs_half(x)
    assert y["a"].dtype == torch.float16 and y["b"][0].dtype == torch.int64 and y["b"][1].dtype == torch.float16


def _api(out):
    import deepspeedsyclsupport_amd as ds
    eng, *_ = ds.initialize(model=_net(), config=_cfg(zero_optimization={"stage": 2, "reduce_bucket_size": 12345},
                                                      gradient_accumulation_steps=2))
    res = {}
    res["batch_info"] = eng.get_batch_info()
    res["bucket"] = eng.zero_reduce_bucket_size()
    res["names"] = (eng.optimizer_name(), eng.scheduler_name(), eng.zero_cpu_offload(), eng.zero_has_nvme_offload(),
                    eng.dynamic_loss_scale(), eng.postscale_gradients(), eng.zero_quantized_nontrainable_weights())
    res["types"] = [str(t) for t in eng.get_data_types()]
    applied = []
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        x, y = torch.randn(2, H, generator=g), torch.randint(0, 4, (2, ), generator=g)
        eng.backward(nn.functional.cross_entropy(eng(x), y))
        eng.step()
        applied.append(eng.was_step_applied())
    res["applied"] = applied
    w = {k: v.clone() + 1.0 for k, v in eng.module.state_dict().items()}
    eng.load_module_state_dict({"module": w})
    res["loaded"] = all(torch.equal(v, w[k]) for k, v in eng.module.state_dict().items())
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    p = next(eng.module.parameters())
    res["master_follows"] = bool(torch.equal(safe_get_full_fp32_param(p).cpu(), w["0.weight"]))
    eng.set_train_micro_batch_size(4)
    res["batch_info2"] = eng.get_batch_info()
    eng.update_optimizer_step(7)
    eng.empty_partition_cache()
    eng.destroy()
    torch.save(res, out)


def test_engine_api_surface(tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_api, 1, out)
    r = torch.load(out)
    assert r["batch_info"] == (4, 2, 2) and r["batch_info2"] == (8, 4, 2)
    assert r["bucket"] == 12345
    assert r["names"] == ("adamw", None, False, False, True, True, False)
    assert r["types"] == ["torch.float32", "torch.float32"]
    assert r["applied"] == [False, True, False, True]
    assert r["loaded"] and r["master_follows"]


def _zero_keys(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.zero.utils import ZeRORuntimeException
    res = {}
    # reduce_scatter: false -> all-reduce + slice; same numbers as the reduce-scatter run
    runs = {}
    for rs in (True, False):
        eng, *_ = ds.initialize(model=_net(), config=_cfg(zero_optimization={"stage": 2, "reduce_scatter": rs,
                                                                             "overlap_comm": False}))
        calls = {"rs": 0, "ar": 0}
        o_rs, o_ar = dist.reduce_scatter_tensor, dist.all_reduce

        def c_rs(*a, **k):
            calls["rs"] += 1
            return o_rs(*a, **k)

        def c_ar(*a, **k):
            calls["ar"] += 1
            return o_ar(*a, **k)

        dist.reduce_scatter_tensor, dist.all_reduce = c_rs, c_ar
        losses = _steps(eng, 3, seed=3 + dist.get_rank())
        dist.reduce_scatter_tensor, dist.all_reduce = o_rs, o_ar
        runs[rs] = (losses, dict(calls), eng.optimizer.rs_stream is None)
    res["runs"] = runs
    # ignore_unused_parameters: false -> a parameter that gets no gradient is an error
    class Unused(nn.Module):

        def __init__(self):
            super().__init__()
            self.a, self.b = nn.Linear(H, 4), nn.Linear(H, 4)

        def forward(self, x):
            return self.a(x)

    eng, *_ = ds.initialize(model=Unused(), config=_cfg(zero_optimization={"stage": 2,
                                                                           "ignore_unused_parameters": False}))
    x, y = torch.randn(2, H), torch.randint(0, 4, (2, ))
    try:
        eng.backward(nn.functional.cross_entropy(eng(x), y))
        res["unused_raised"] = False
    except ZeRORuntimeException as e:
        res["unused_raised"] = "ignore_unused_parameters" in str(e)
    # model_persistence_threshold caps what stays gathered under ZeRO-3
    for cap in (None, 40):
        z = {"stage": 3, "stage3_param_persistence_threshold": 1000}
        if cap is not None:
            z["stage3_model_persistence_threshold"] = cap
        eng, *_ = ds.initialize(model=_net(), config=_cfg(zero_optimization=z))
        res[f"persistent_{cap}"] = sum(g.numel for g in eng.optimizer.groups if g.persistent)
    if dist.get_rank() == 0:
        torch.save(res, out)


def test_zero_keys_change_behaviour(tmp_path):
    out = str(tmp_path / "r.pt")
    run_distributed(_zero_keys, 2, out)
    r = torch.load(out)
    (l1, c1, nostream1), (l0, c0, nostream0) = r["runs"][True], r["runs"][False]
    assert l1 == pytest.approx(l0, rel=1e-6) and c1["rs"] > 0 and c0["rs"] == 0 and c0["ar"] > c1["ar"]
    assert nostream1 and nostream0       # overlap_comm: false was spelled out (no side streams on CPU anyway)
    assert r["unused_raised"]
    assert r["persistent_40"] < r["persistent_None"] and r["persistent_40"] <= 40 + 16
