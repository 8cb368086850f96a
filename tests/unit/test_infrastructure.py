"""Accelerator, op-builder registry, environment report, batch-size solving, process groups, collectives facade, timers
and the native async I/O handle (reference `tests/unit/accelerator`, `tests/unit/ops/accelerators`,
`tests/unit/runtime/test_ds_config_dict.py`, `tests/unit/utils/test_groups.py`, `tests/unit/comm/test_dist.py`,
`tests/unit/ops/aio/test_aio.py`)."""
import os

import pytest
import torch

from .common import run_distributed


# ----------------------------------------------------------------------------------------------- accelerator
def test_accelerator_surface():
    from deepspeedsyclsupport_amd.accelerator import get_accelerator
    acc = get_accelerator()
    assert acc.communication_backend_name() in ("nccl", "gloo")
    assert acc.device_name() in ("cuda", "cpu") and acc.device_count() >= 0
    assert torch.bfloat16 in acc.supported_dtypes() or not acc.is_bf16_supported()
    acc.manual_seed(7)
    state = acc.get_rng_state()
    acc.set_rng_state(state)
    acc.range_push("x")
    acc.range_pop()
    acc.synchronize()
    s, e = acc.Stream(), acc.Event()
    assert s is not None and e is not None
    with acc.stream(s):
        t = torch.ones(4)
    assert acc.on_accelerator(t) == (t.device.type == acc.device_name())
    assert acc.memory_allocated() >= 0 and acc.total_memory() >= 0
    pinned = acc.pin_memory(torch.zeros(8)) if acc.device_name() == "cuda" else torch.zeros(8)
    assert pinned.numel() == 8
    assert os.path.isdir(os.path.dirname(acc.op_builder_dir().replace(".", "/"))) or isinstance(acc.op_builder_dir(), str)


# ----------------------------------------------------------------------------------------------- op builders
def test_every_reference_builder_name_resolves():
    from deepspeedsyclsupport_amd.ops import op_builder
    names = {"fused_adam", "cpu_adam", "cpu_adagrad", "cpu_lion", "fused_lion", "fused_lamb", "quantizer",
             "random_ltd", "transformer", "stochastic_transformer", "transformer_inference", "spatial_inference",
             "sparse_attn", "async_io", "evoformer_attn", "inference_core_ops", "cutlass_ops", "ragged_device_ops",
             "ragged_ops", "deepspeed_ccl_comm", "utils"}
    assert names <= set(op_builder.ALL_OPS), sorted(names - set(op_builder.ALL_OPS))
    for name in names:
        b = op_builder.ALL_OPS[name]()
        assert name in b.absolute_name()
        assert isinstance(b.is_compatible(), bool)
    mod = op_builder.ALL_OPS["cpu_adam"]().load()
    assert hasattr(mod, "adam_update") or hasattr(mod, "cpu_adam_update")
    assert op_builder.is_built("ds_cpu_ops") and op_builder.is_built("ds_hip_ops")


def test_env_report_lists_ops(capsys):
    from deepspeedsyclsupport_amd import env_report
    env_report.main()
    out = capsys.readouterr().out
    for needle in ("fused_adam", "async_io", "torch version", "target arch", "distributed backends"):
        assert needle in out


# ----------------------------------------------------------------------------------------------- config
@pytest.mark.parametrize("given,world,want", [
    ({"train_batch_size": 32, "train_micro_batch_size_per_gpu": 2}, 4, (32, 2, 4)),
    ({"train_batch_size": 32, "gradient_accumulation_steps": 2}, 4, (32, 4, 2)),
    ({"train_micro_batch_size_per_gpu": 3, "gradient_accumulation_steps": 5}, 2, (30, 3, 5)),
    ({"train_batch_size": 16}, 4, (16, 4, 1)),
    ({"train_micro_batch_size_per_gpu": 8}, 2, (16, 8, 1)),
])
def test_batch_triple_is_solved(given, world, want):
    from deepspeedsyclsupport_amd.runtime.config import DeepSpeedConfig

    class _MPU:

        def get_data_parallel_world_size(self):
            return world

    c = DeepSpeedConfig(dict(given), mpu=_MPU())
    assert (c.train_batch_size, c.train_micro_batch_size_per_gpu, c.gradient_accumulation_steps) == want


def test_inconsistent_batch_triple_raises():
    from deepspeedsyclsupport_amd.runtime.config import DeepSpeedConfig, DeepSpeedConfigError

    class _MPU:

        def get_data_parallel_world_size(self):
            return 2

    with pytest.raises((DeepSpeedConfigError, AssertionError, ValueError)):
        DeepSpeedConfig({"train_batch_size": 10, "train_micro_batch_size_per_gpu": 3,
                         "gradient_accumulation_steps": 1}, mpu=_MPU())
    with pytest.raises((DeepSpeedConfigError, AssertionError, ValueError)):
        DeepSpeedConfig({}, mpu=_MPU())


def test_config_from_json_path_and_zero_defaults(tmp_path):
    import json

    from deepspeedsyclsupport_amd.runtime.config import DeepSpeedConfig
    p = tmp_path / "ds.json"
    p.write_text(json.dumps({"train_batch_size": 4, "zero_optimization": {"stage": 3}, "bf16": {"enabled": True}}))
    c = DeepSpeedConfig(str(p))
    z = c.zero_config
    assert c.zero_optimization_stage == 3 and c.bfloat16_enabled
    assert z.reduce_bucket_size > 0 and z.prefetch_bucket_size > 0 and z.param_persistence_threshold > 0


# ----------------------------------------------------------------------------------------------- groups
def _groups():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.parallel import groups
    ds.init_distributed(dist_backend="gloo")
    r = dist.get_rank()
    groups.reset()
    groups._create_expert_and_data_parallel(2)
    name = "ep_size_2"
    assert groups._get_expert_parallel_world_size(name) == 2 and groups._get_expert_data_parallel_world_size(name) == 2
    # E + D: expert-parallel groups are consecutive ranks, expert-data groups stride over them
    assert groups._get_expert_parallel_rank(name) == r % 2 and groups._get_expert_data_parallel_rank(name) == r // 2
    t = torch.tensor([float(r)])
    dist.all_reduce(t, group=groups._get_expert_parallel_group(name))
    assert float(t) == {0: 1.0, 1: 1.0, 2: 5.0, 3: 5.0}[r]
    t = torch.tensor([float(r)])
    dist.all_reduce(t, group=groups._get_expert_data_parallel_group(name))
    assert float(t) == {0: 2.0, 2: 2.0, 1: 4.0, 3: 4.0}[r]
    assert groups._get_data_parallel_world_size() == 4
    groups._create_zero_param_parallel_group(2)  # hpZ secondary groups of consecutive ranks
    assert groups._get_zero_param_intra_parallel_group_world_size() == 2
    assert groups._get_zero_param_intra_parallel_group_ranks() == [r - r % 2, r - r % 2 + 1]
    groups.initialize_sequence_parallel(2)
    assert groups._get_sequence_parallel_world_size() == 2 and groups._get_sequence_parallel_rank() == r % 2
    assert groups._get_sequence_data_parallel_world_size() == 4


def test_expert_hpz_and_sequence_groups_world4():
    run_distributed(_groups, 4)


# ----------------------------------------------------------------------------------------------- collectives facade
def _collectives():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    ds.init_distributed(dist_backend="gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    dist.configure(enabled=True, prof_all=True, verbose=False)
    x = torch.full((4, ), float(r + 1))
    dist.all_reduce(x)
    assert x.tolist() == [6.0] * 4
    out = torch.empty(2 * w)
    dist.all_gather_into_tensor(out, torch.full((2, ), float(r)))
    assert out.tolist() == [0.0, 0.0, 1.0, 1.0, 2.0, 2.0]
    rs = torch.empty(2)
    dist.reduce_scatter_tensor(rs, torch.arange(2 * w, dtype=torch.float32))
    assert rs.tolist() == [3.0 * (2 * r), 3.0 * (2 * r + 1)]
    a2a = torch.empty(w)
    dist.all_to_all_single(a2a, torch.full((w, ), float(r)))
    assert a2a.tolist() == [0.0, 1.0, 2.0]
    b = torch.tensor([float(r)])
    dist.broadcast(b, src=2)
    assert float(b) == 2.0
    if r == 0:
        dist.send(torch.tensor([42.0]), dst=1)
    elif r == 1:
        got = torch.zeros(1)
        dist.recv(got, src=0)
        assert float(got) == 42.0
    dist.barrier()
    assert dist.get_world_group() is not None and dist.get_local_rank() >= 0
    summary = dist.log_summary(show_straggler=False)
    logged = dist.comms_logger.comms_dict if hasattr(dist, "comms_logger") else summary
    assert logged is None or "all_reduce" in str(logged)


def test_collectives_and_comms_logger_world3():
    run_distributed(_collectives, 3)


# ----------------------------------------------------------------------------------------------- timers
def test_wall_clock_and_throughput_timers():
    from deepspeedsyclsupport_amd.utils.timer import SynchronizedWallClockTimer, ThroughputTimer
    timers = SynchronizedWallClockTimer()
    timers("fwd").start()
    sum(range(10000))
    timers("fwd").stop()
    assert timers("fwd").elapsed(reset=False) >= 0.0
    means = timers.get_mean(["fwd"], reset=True)
    assert "fwd" in means
    tp = ThroughputTimer(batch_size=8, start_step=1, steps_per_output=1000)
    for _ in range(3):
        tp.start()
        tp.stop(global_step=True)
    assert tp.avg_samples_per_sec() > 0


# ----------------------------------------------------------------------------------------------- async I/O
def test_aio_handle_round_trip(tmp_path):
    from deepspeedsyclsupport_amd.ops.aio import AsyncIOBuilder
    aio = AsyncIOBuilder().load()
    h = aio.aio_handle(block_size=128 * 1024, queue_depth=8, single_submit=False, overlap_events=True, num_threads=2)
    assert h.get_block_size() == 128 * 1024 and h.get_queue_depth() == 8 and h.get_thread_count() == 2
    src = h.new_cpu_locked_tensor(1 << 18, torch.empty(0, dtype=torch.float32))
    src.copy_(torch.arange(1 << 18, dtype=torch.float32))
    path = str(tmp_path / "t.bin")
    assert h.sync_pwrite(src, path) >= 0
    dst = h.new_cpu_locked_tensor(1 << 18, torch.empty(0, dtype=torch.float32))
    dst.zero_()
    h.async_pread(dst, path)
    assert h.wait() == 1
    assert torch.equal(dst, src)
    assert os.path.getsize(path) == (1 << 18) * 4
    h.free_cpu_locked_tensor(src)
    h.free_cpu_locked_tensor(dst)


def test_reference_import_paths_resolve():
    """Module paths of the reference that are folded into other files here still import (served by the package's
    import-path finder) and hand out the real classes."""
    import importlib

    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import _import_paths
    from deepspeedsyclsupport_amd.runtime.zero.flat_optimizer import FlatZeroOptimizer
    for rel, targets in _import_paths.PATHS.items():
        mod = importlib.import_module(f"deepspeedsyclsupport_amd.{rel}")
        for _, names in targets:
            if names != "*":
                for exposed in names:
                    assert hasattr(mod, exposed), (rel, exposed)
    from deepspeedsyclsupport_amd.accelerator.real_accelerator import get_accelerator
    from deepspeedsyclsupport_amd.runtime.zero.stage3 import DeepSpeedZeroOptimizer_Stage3
    assert issubclass(DeepSpeedZeroOptimizer_Stage3, FlatZeroOptimizer) and get_accelerator is ds.get_accelerator
    with pytest.raises(ModuleNotFoundError):
        importlib.import_module("deepspeedsyclsupport_amd.runtime.zero.no_such_module")


def test_accelerator_builder_and_legacy_surface():
    """Names of the reference accelerator ABC that integrations call (`accelerator/abstract_accelerator.py`): op
    builder lookup, legacy tensor constructors, older memory-stat names."""
    import torch

    from deepspeedsyclsupport_amd.accelerator import get_accelerator
    a = get_accelerator()
    b = a.create_op_builder("FusedAdamBuilder")
    assert b is not None and type(b) is a.get_op_builder("FusedAdamBuilder") and a.get_op_builder("NoSuchBuilder") is None
    assert a.FloatTensor([1, 2]).dtype == torch.float32 and a.HalfTensor([1]).dtype == torch.float16
    assert a.LongTensor([1]).dtype == torch.int64 and a.BFloat16Tensor([1]).dtype == torch.bfloat16
    assert a.memory_cached() == a.memory_reserved() and a.max_memory_cached() == a.max_memory_reserved()
    assert a.amp() is torch.amp and not a.is_triton_supported() and "RCCL" in a.export_envs()


def test_config_key_constants_follow_the_defaults_tables():
    """`compression.constants` is built from the defaults tables the config parser uses; the data-pipeline key
    names are served under the reference's path."""
    from deepspeedsyclsupport_amd.compression import constants as cc
    from deepspeedsyclsupport_amd.compression.config import SHARED_DEFAULTS
    from deepspeedsyclsupport_amd.runtime.data_pipeline import constants as dc
    assert cc.WEIGHT_QUANTIZATION == "weight_quantization" and cc.WEIGHT_QUANTIZE_GROUPS == "quantize_groups"
    assert cc.WEIGHT_QUANTIZE_GROUPS_DEFAULT == SHARED_DEFAULTS["weight_quantization"]["quantize_groups"]
    assert cc.WEIGHT_QUANTIZE_STOCHASTIC_ROUNDING == "stochastic" and cc.ACTIVATION_QUANTIZE_RANGE_STATIC == "static"
    assert cc.SPARSE_PRUNING_METHOD_SNIP_MOMENTUM == "snip_momentum" and cc.HEAD_PRUNING_NUM_HEADS == "num_heads"
    assert cc.KEEP_NUMBER_LAYER == "keep_number_layer"
    assert dc.RANDOM_LTD_SCHEDULER == "random_ltd_schedule" and dc.RANDOM_LTD_ENABLED_DEFAULT is False
    assert dc.CURRICULUM_LEARNING_SCHEDULE_FIXED_ROOT == "fixed_root" and dc.DATA_EFFICIENCY_SEED_DEFAULT == 1234
