"""Small runtime parts with reference counterparts: the defragmenting contiguous allocator
(`runtime/zero/contiguous_memory_allocator.py`), swap-buffer pools (`runtime/swap_tensor/utils.py`), pipeline p2p
object transfer (`runtime/pipe/p2p.py`), the autotuning config section and the served reference import paths."""
import importlib

import pytest
import torch

from ..common import run_distributed


def test_contiguous_allocator_defragments_and_keeps_params():
    from deepspeedsyclsupport_amd.runtime.zero.contiguous_memory_allocator import ContiguousMemoryAllocator
    mem = ContiguousMemoryAllocator(100, torch.float32, "cpu")
    a, b, c = mem.allocate_tensor(30), mem.allocate_tensor(30), mem.allocate_tensor(30)
    a.fill_(1), b.fill_(2), c.fill_(3)
    p = torch.nn.Parameter(torch.empty(0))
    mem.assign_to_param(c, p, 24, (4, 6))
    assert p.data.shape == (4, 6) and float(p.data.sum()) == 72
    mem.release_tensor(b)
    assert mem.total_free == 40 and mem.largest_contiguous == 30
    d = mem.allocate_tensor(40)          # needs the two holes merged: c slides down next to a
    d.fill_(4)
    assert mem.total_free == 0 and float(a.sum()) == 30 and float(c.sum()) == 90 and float(p.data.sum()) == 72
    assert p.data.data_ptr() == c.data_ptr() and mem.max_allocated_size() == 100
    c.add_(1)                            # the parameter still aliases the moved tensor
    assert float(p.data.sum()) == 96
    with pytest.raises(MemoryError):
        mem.allocate_tensor(1)
    mem.release_tensor(a)
    with pytest.raises(ValueError):
        mem.release_tensor(a)


def test_swap_buffer_pool(tmp_path):
    from deepspeedsyclsupport_amd.runtime.swap_tensor.utils import (SwapBufferManager, SwapBufferPool,
                                                                    get_aligned_numel)
    assert get_aligned_numel(1000, 4) == 1024 and get_aligned_numel(256, 4) == 256
    mgr = SwapBufferManager(num_elems=1024, count=3, dtype=torch.float32)
    bufs = mgr.allocate(1024, 2, torch.float32)
    assert len(bufs) == 2 and mgr.allocate(1024, 2, torch.float32) is None
    pool = SwapBufferPool(bufs)
    t1, t2 = torch.arange(600.), torch.arange(700.)
    s1, c1 = pool.insert_tensor(t1, str(tmp_path / "a"), 768)
    s2, c2 = pool.insert_tensor(t2, str(tmp_path / "b"), 768)   # does not fit beside t1: goes to the second slice
    assert s1.numel() == 768 and torch.equal(c1, t1) and torch.equal(c2, t2) and pool.current_index == 1
    assert pool.insert_tensor(torch.zeros(600), "c", 768) == (None, None)
    assert pool.get_swap_paths() == [str(tmp_path / "a"), str(tmp_path / "b")]
    mgr.free(bufs)
    assert len(mgr.allocate_all(512, torch.float32)) == 3


def _p2p_objects():
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.pipe import p2p
    from deepspeedsyclsupport_amd.runtime.pipe.topology import PipeDataParallelTopology, PipelineParallelGrid
    dist.init_distributed("gloo")
    grid = PipelineParallelGrid(topology=PipeDataParallelTopology(num_pp=2, num_dp=1))
    p2p.init_process_groups(grid)
    msg = {"shape": (2, 3), "parts": [torch.arange(6).view(2, 3), "tag"], "n": 7}
    if grid.get_stage_id() == 0:
        p2p.send_obj(msg, 1)
        p2p.send(torch.full((4, ), 5.0), 1)
    else:
        got = p2p.recv_obj(0)
        assert got["shape"] == (2, 3) and got["n"] == 7 and got["parts"][1] == "tag"
        assert torch.equal(got["parts"][0], torch.arange(6).view(2, 3))
        buf = torch.zeros(4)
        p2p.recv(buf, 0)
        assert buf.tolist() == [5.0] * 4
    p2p.wait()


def test_pipe_p2p_objects():
    run_distributed(_p2p_objects, 2)


def test_autotuning_config_validation():
    from deepspeedsyclsupport_amd.autotuning.config import DeepSpeedAutotuningConfig
    c = DeepSpeedAutotuningConfig({"autotuning": {"enabled": True, "tuner_type": "random", "fast": False}})
    assert c.enabled and c.tuner_type == "random" and not c.fast and c.results_dir == "autotuning_results"
    with pytest.raises(Exception):
        DeepSpeedAutotuningConfig({"autotuning": {"tuner_typ": "random"}})


@pytest.mark.parametrize("path,names", [
    ("inference.v2.kernels.ragged_ops.blocked_flash.blocked_flash", ["BlockedFlashAttn", "get_q_block_size"]),
    ("inference.v2.kernels.core_ops.cuda_rms_norm.rms_pre_norm", ["CUDARMSPreNorm"]),
    ("inference.v2.modules.interfaces.attention_base", ["DSSelfAttentionBase", "DSSelfAttentionRegistry"]),
    ("inference.v2.modules.implementations.moe.cutlass_multi_gemm", ["DSMultiGemmMoE"]),
    ("inference.v2.model_implementations.llama_v2.policy", ["Llama2Policy"]),
    ("inference.v2.model_implementations.mixtral.container", ["MixtralTransformerContainer"]),
    ("inference.v2.model_implementations.sharding.qkv", ["shard_qkv_param"]),
    ("inference.v2.ragged.ragged_wrapper", ["RaggedBatchWrapper"]),
    ("runtime.comm.nccl", ["NcclBackend"]),
    ("runtime.swap_tensor.partitioned_param_swapper", ["AsyncPartitionedParameterSwapper"]),
    ("model_implementations.transformers.ds_transformer", ["DeepSpeedTransformerInference"]),
    ("ops.deepspeed4science.evoformer_attn", ["DS4Sci_EvoformerAttention"]),
    ("runtime.pipe.p2p", ["send_obj", "recv_obj"]),
    ("monitor.utils", ["check_tb_availability"]),
    ("nebula.config", ["DeepSpeedNebulaConfig"]),
    ("git_version_info", ["version", "installed_ops"]),
])
def test_reference_paths_resolve(path, names):
    mod = importlib.import_module("deepspeedsyclsupport_amd." + path)
    for n in names:
        assert hasattr(mod, n), (path, n)


def test_generated_constants_follow_the_config_models():
    cc = importlib.import_module("deepspeedsyclsupport_amd.comm.constants")
    assert cc.COMMS_LOGGER == "comms_logger" and cc.COMMS_LOGGER_ENABLED == "enabled"
    assert cc.COMMS_LOGGER_ENABLED_DEFAULT is False and cc.NCCL_BACKEND == "nccl"
    ac = importlib.import_module("deepspeedsyclsupport_amd.autotuning.constants")
    assert ac.AUTOTUNING_TUNER_TYPE == "tuner_type" and ac.AUTOTUNING_TUNER_TYPE_DEFAULT == "gridsearch"
    ec = importlib.import_module("deepspeedsyclsupport_amd.elasticity.constants")
    assert ec.MICRO_BATCHES == "micro_batch_sizes" and ec.LATEST_ELASTICITY_VERSION == 0.2


def test_quantization_context_quantizes_modules_built_inside():
    from deepspeedsyclsupport_amd.inference.quantization.layers import QuantizedLinear
    from deepspeedsyclsupport_amd.inference.quantization.quantization_context import QuantizationContext
    cfg = {"weight_quantization": {"quantized_initialization": {"num_bits": 8, "group_size": 32, "group_dim": 1,
                                                                  "symmetric": False}}}
    before = torch.nn.Module.__init__
    with QuantizationContext(config_dict_or_path=cfg):
        net = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, 32))
    assert torch.nn.Module.__init__ is before
    assert isinstance(net[0], QuantizedLinear) and isinstance(net[2], QuantizedLinear)
    assert net(torch.randn(3, 64)).shape == (3, 32)


def _ccl_backend():
    from deepspeedsyclsupport_amd.comm.ccl import CCLBackend
    be = CCLBackend()
    assert be.is_initialized() and be.world_size == 2 and "inference_all_reduce" in be.available_coll
    t = torch.full((5, ), float(be.world_rank + 1))
    be.all_reduce(t)
    assert t.tolist() == [3.0] * 5
    t = torch.full((1024, ), float(be.world_rank + 1))
    be.inference_all_reduce(t)          # host tensors: the shared-memory reduce when the native extension is there
    assert t.tolist() == [3.0] * 1024
    b = torch.arange(4.) if be.world_rank == 0 else torch.zeros(4)
    be.broadcast(b, 0)
    assert b.tolist() == [0.0, 1.0, 2.0, 3.0]
    be.barrier()


def test_ccl_backend_object():
    run_distributed(_ccl_backend, 2)


def test_memory_estimators_and_runtime_helpers(capsys):
    from deepspeedsyclsupport_amd.runtime import utils as U
    from deepspeedsyclsupport_amd.runtime.zero.stage3 import (estimate_zero3_model_states_mem_needs,
                                                           estimate_zero3_model_states_mem_needs_all_live)
    from deepspeedsyclsupport_amd.runtime.zero.stage_1_and_2 import estimate_zero2_model_states_mem_needs
    P, L = 10**9, 10**8
    cpu, gpu = estimate_zero2_model_states_mem_needs(P, 8, 1, cpu_offload=False)
    assert gpu == 4 * P + 16 * P // 8
    cpu, gpu, big = estimate_zero3_model_states_mem_needs(P, L, 8, 2, cpu_offload=False)
    assert gpu == 4 * L + 18 * P // 16 and big == 4 * L
    cpu, gpu, _ = estimate_zero3_model_states_mem_needs(P, L, 8, 1, cpu_offload=True, cpu_offload_params=True)
    assert gpu == 4 * L and cpu == int(P * 18 * 1.5)
    rows = estimate_zero3_model_states_mem_needs_all_live(torch.nn.Linear(100, 100), 2, 1)
    assert len(rows) == 6 and "largest layer params" in capsys.readouterr().out
    ts = [torch.full((4, ), 3.0), torch.full((9, ), 2.0)]
    before = U.clip_tensors_by_global_norm(ts, 1.0)
    assert abs(float(before) - 72**0.5) < 1e-4 and abs(float(U.get_global_norm_of_tensors(ts)) - 1.0) < 1e-4
    assert U.get_global_norm([3, 4]) == 5.0 and U.prefix_sum_inc([1, 2, 3]) == [1, 3, 6]
    moved = U.copy_to_device({"a": [ts[0]], "b": 1}, "cpu")
    assert moved["a"][0] is not ts[0] and torch.equal(moved["a"][0], ts[0]) and moved["b"] == 1


def _local_fragments():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.utils.tensor_fragment import (safe_get_full_fp32_param,
                                                               safe_get_local_fp32_param,
                                                               safe_get_local_optimizer_state,
                                                               safe_set_local_fp32_param,
                                                               safe_set_local_optimizer_state)
    from unit.simple_model import base_config, random_tokens, tiny_llama
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=base_config(stage=3, lr=1e-2, mb=2))
    x = random_tokens(1, 2, 16, seed=1)[0]
    eng.backward(eng(x, labels=x))
    eng.step()
    p = next(q for n, q in eng.module.named_parameters() if "q_proj" in n or "qkv" in n)
    local = safe_get_local_fp32_param(p)           # None on a rank whose partition holds nothing of p
    if local is not None:
        safe_set_local_fp32_param(p, torch.full_like(local, 0.25))
    full = safe_get_full_fp32_param(p)
    assert torch.all(full == 0.25)                 # every owning rank wrote its own fragment
    m = safe_get_local_optimizer_state(p, "exp_avg")
    if m is not None:
        safe_set_local_optimizer_state(p, torch.ones_like(m), "exp_avg")
        assert torch.all(safe_get_local_optimizer_state(p, "exp_avg") == 1)
        with pytest.raises(ValueError):
            safe_set_local_fp32_param(p, torch.zeros(local.numel() + 1))


def test_local_fragment_setters_zero3():
    run_distributed(_local_fragments, 2)


def test_legacy_indexed_dataset_formats(tmp_path):
    """The pre-mmap index format ("lazy" / "cached" readers, builder, merge) next to the mmap one."""
    import numpy as np

    from deepspeedsyclsupport_amd.runtime.data_pipeline.data_sampling import indexed_dataset as I
    base = str(tmp_path / "legacy")
    items = [np.arange(5), np.arange(3) + 10, np.arange(7) + 100]
    b = I.make_builder(I.data_file_path(base), impl="cached", dtype=np.int32)
    for it in items:
        b.add_item(torch.tensor(it))
    b.end_document()
    b.finalize(I.index_file_path(base))
    assert I.infer_dataset_impl(base) == "cached" and I.dataset_exists(base, "lazy")
    ds = I.make_dataset(base, "infer")
    assert isinstance(ds, I.IndexedCachedDataset) and len(ds) == 3 and ds.doc_idx.tolist() == [0, 3]
    ds.prefetch([0, 2])
    assert ds[2].tolist() == items[2].tolist() and ds[1].tolist() == items[1].tolist()
    lazy = I.make_dataset(base, "lazy")
    assert [x.tolist() for x in lazy[0:2]] == [items[0].tolist(), items[1].tolist()]
    other = str(tmp_path / "other")
    b2 = I.IndexedDatasetBuilder(I.data_file_path(other), dtype=np.int32)
    b2.add_item(torch.tensor([7, 8]))
    b2.merge_file_(base)
    b2.finalize(I.index_file_path(other))
    merged = I.IndexedDataset(other)
    assert len(merged) == 4 and merged[3].tolist() == items[2].tolist() and merged[0].tolist() == [7, 8]
    ptr, total = I.get_pointers_with_total([2, 3, 4], 4, np.int64)
    assert ptr.tolist() == [0, 8, 20] and total == 36 and I.create_doc_idx([3, 0, 2, 0]) == [0, 2, 4]
    assert I.get_available_dataset_impl() == ["lazy", "cached", "mmap"]
