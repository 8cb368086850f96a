"""Engine options that change how gradients are reduced or data is fed (reference `runtime/engine.py:325-327,
1144-1145,1723-1740,2331-2341,2447-2518`, `runtime/dataloader.py:60-89`), on gloo with 2 ranks:

* `prescale_gradients` / `gradient_predivide_factor`: same update as the default post-scaled average, while the
  factor actually applied before the collective is the configured one;
* `sparse_gradients`: embedding gradients all-gathered as (row indices, rows) train exactly like the dense reduction;
* `seq_parallel_communication_data_type`: the reduction dtype under Ulysses;
* curriculum learning through `engine.deepspeed_io`: batches only contain samples the scheduler allows.
"""
import numpy as np
import pytest
import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama


def _train(extra, out, stage, check=None):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    cfg = base_config(stage=stage, lr=1e-2, mb=2, clip=1.0)
    cfg.update(extra)
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    losses = []
    for x in random_tokens(3, 2, 16, seed=11 + dist.get_rank()):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    if check:
        check(eng)
    w = {n: safe_get_full_fp32_param(p) for n, p in eng.module.named_parameters()}
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "w": w}, out)


def _same(tmp_path, stage, extra, check=None, rtol=1e-5, atol=1e-6):
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    run_distributed(_train, 2, {}, a, stage)
    run_distributed(_train, 2, extra, b, stage, check)
    ref, got = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    assert got["losses"] == pytest.approx(ref["losses"], rel=1e-5, abs=1e-6)
    for n in ref["w"]:
        torch.testing.assert_close(got["w"][n], ref["w"][n], rtol=rtol, atol=atol, msg=n)


def _check_predivide(eng):
    opt = eng.optimizer
    g = opt.groups[0]
    assert opt._pre_factor(g) == pytest.approx(1.0 / 4.0) and opt._alpha(g) == pytest.approx(4.0 / 2.0)


def _check_prescale(eng):
    opt = eng.optimizer
    g = opt.groups[0]
    assert opt._pre_factor(g) == pytest.approx(0.5) and opt._alpha(g) == pytest.approx(1.0)


@pytest.mark.parametrize("stage", [0, 2, 3])
def test_gradient_predivide_factor(stage, tmp_path):
    _same(tmp_path, stage, {"gradient_predivide_factor": 4.0}, _check_predivide)


@pytest.mark.parametrize("stage", [0, 2])
def test_prescale_gradients(stage, tmp_path):
    _same(tmp_path, stage, {"prescale_gradients": True}, _check_prescale)


def _check_sparse(eng):
    assert "model.embed_tokens.weight" in eng.sparse_tensor_module_names
    opt = eng.optimizer
    assert opt.sparse_reductions == 3 and sum(1 for g in opt.groups if g.sparse) == 1


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_sparse_embedding_gradients(stage, tmp_path):
    # (rows summed after an all-gather vs inside a reduce-scatter: a different fp32 summation order)
    _same(tmp_path, stage, {"sparse_gradients": True}, _check_sparse, atol=5e-6)


def test_sparse_tensor_allreduce_roundtrip():
    """SparseTensor keeps only touched rows; to_dense restores the gradient (reference `runtime/sparse_tensor.py`)."""
    from deepspeedsyclsupport_amd.runtime.sparse_tensor import SparseTensor
    g = torch.zeros(50, 8)
    g[[3, 17, 41]] = torch.randn(3, 8)
    st = SparseTensor(g)
    assert sorted(st.indices.tolist()) == [3, 17, 41] and st.sparse_size()[0] == 3 + 24
    torch.testing.assert_close(st.to_dense(), g)


def _sp_comm_dtype(dtype_key, out):
    import deepspeedsyclsupport_amd as ds
    cfg = base_config(stage=2, lr=1e-2, mb=2, dtype="bf16")
    cfg["sequence_parallel"] = {"size": 2}
    cfg["train_batch_size"] = 2
    if dtype_key:
        cfg["seq_parallel_communication_data_type"] = dtype_key
    eng, _, _, _ = ds.initialize(model=tiny_llama(num_attention_heads=4), config=cfg)
    want = {"bf16": torch.bfloat16, None: torch.float32, "fp32": torch.float32}[dtype_key]
    assert eng.optimizer.comm_dtype == want, (eng.optimizer.comm_dtype, want)
    x = random_tokens(1, 2, 16, seed=3)[0]
    loss = eng(x[:, :8] if ds.comm.get_rank() == 0 else x[:, 8:], labels=None)
    assert loss is not None


@pytest.mark.parametrize("dtype_key", [None, "bf16"])
def test_seq_parallel_communication_data_type(dtype_key, tmp_path):
    run_distributed(_sp_comm_dtype, 2, dtype_key, None)


class _Toy(torch.utils.data.Dataset):

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return torch.tensor([i, i % 7])


def _curriculum(metric_path, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.data_pipeline.data_sampling.data_sampler import DeepSpeedDataSampler
    cfg = base_config(stage=1, lr=1e-2, mb=4, gas=2)
    cfg["data_efficiency"] = {
        "enabled": True, "seed": 7,
        "data_sampling": {"enabled": True, "num_workers": 0, "curriculum_learning": {
            "enabled": True, "curriculum_metrics": {"difficulty": {
                "sample_to_metric_path": metric_path, "difficulty_type": "value", "min_difficulty": 10,
                "max_difficulty": 100, "schedule_type": "fixed_linear",
                "schedule_config": {"total_curriculum_step": 4, "difficulty_step": 10}}}}}}
    ds_ = _Toy(100)
    eng, _, loader, _ = ds.initialize(model=tiny_llama(), config=cfg, training_data=ds_)
    assert eng.curriculum_learning_enabled() and isinstance(loader.data_sampler, DeepSpeedDataSampler)
    assert loader.curriculum_learning_enabled
    metric = np.load(metric_path)
    seen = []
    it = iter(loader)
    for step in range(1, 5):
        for _ in range(2):  # gas micro-batches of one global batch share the step's difficulty
            batch = next(it)
            assert batch.shape == (4, 2)
            ids = batch[:, 0].tolist()
            limit = loader.data_sampler.schedulers["difficulty"].get_current_difficulty()
            assert all(metric[i] <= limit for i in ids), (step, ids, limit)
            seen.append(ids)
    # both ranks drew from the same shuffled global batch: their slices are disjoint parts of it
    gathered = [None, None]
    dist.all_gather_object(gathered, seen)
    assert gathered[0] != gathered[1]
    # the sampler state travels in checkpoints
    sd = loader.data_sampler.state_dict()
    assert sd["curriculum_step"] == 4 and sd["consumed_samples"] == 4 * 4 * 2 * 2


def test_curriculum_sampler_through_deepspeed_io(tmp_path):
    path = str(tmp_path / "metric.npy")
    rng = np.random.default_rng(0)
    np.save(path, rng.integers(1, 101, size=100))
    run_distributed(_curriculum, 2, path, None)


def test_dataloader_worker_and_batch_defaults():
    """local_rank >= 0: one process per device, 2 loader workers; local_rank < 0: batch scaled by the device count."""
    from deepspeedsyclsupport_amd.accelerator import get_accelerator
    from deepspeedsyclsupport_amd.runtime.dataloader import DeepSpeedDataLoader
    dl = DeepSpeedDataLoader(_Toy(32), 4, False, 0, None, data_parallel_world_size=1, data_parallel_rank=0)
    assert dl.num_local_io_workers == 2 and dl.batch_size == 4 and dl.device_count == 1
    n = max(get_accelerator().device_count(), 1)
    dl = DeepSpeedDataLoader(_Toy(32), 4, False, -1, None)
    assert dl.batch_size == 4 * n and dl.num_local_io_workers == 2 * n
    dl = DeepSpeedDataLoader(_Toy(32), 4, False, 0, None, num_local_io_workers=0)
    assert len(list(iter(dl))) == 8


def _explicit_reductions(out):
    """`buffered_allreduce_fallback` & co. on module gradients: averages dense grads per dtype bucket and the
    embedding gradient as (indices, rows)."""
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    rank = dist.get_rank()
    cfg = base_config(stage=0, lr=1e-2, mb=2)
    cfg["sparse_gradients"] = True
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    torch.manual_seed(rank)
    grads = {}
    for n, p in eng.module.named_parameters():
        p.grad = torch.randn_like(p)
        if "embed_tokens" in n:
            p.grad[5:] = 0          # only a few rows touched, as an embedding gradient would be
        grads[n] = p.grad.clone()
    every = [None, None]
    dist.all_gather_object(every, grads)
    eng.buffered_allreduce_fallback(elements_per_buffer=1000)    # small buffers: several buckets
    for n, p in eng.module.named_parameters():
        want = (every[0][n] + every[1][n]) / 2
        torch.testing.assert_close(p.grad, want, rtol=1e-5, atol=1e-6, msg=n)
    assert eng.all_gather_scalar(rank + 3) == [3, 4]
    parts = eng.sparse_all_gather(torch.full((rank + 1, 2), float(rank)))
    assert [p.shape[0] for p in parts] == [1, 2] and float(parts[1][0, 0]) == 1.0
    assert eng.is_first_weights_partition_group() and eng.flops_profiler_recompute_fwd_factor() == 0.0


def test_explicit_gradient_reductions(tmp_path):
    run_distributed(_explicit_reductions, 2, None)
