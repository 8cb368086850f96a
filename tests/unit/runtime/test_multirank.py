"""Multi-rank readiness on gloo (no GPU cluster here; the 8-GPU node runs only at round end):

* ZeRO-3 x Ulysses sequence parallel 2 x data parallel 2 (world 4) against a single-process full-sequence reference;
* data parallel 8 ZeRO-3 (world 8) with trace-driven prefetch, qwZ and hpZ against the fp32 single-process reference
  (the exact layout the driver's 8-GPU scaling run uses: dp8, ZeRO-3, every group gathered);
* BASELINE.json config 1: GPT-2 small (124M, HF architecture) ZeRO-1 on the CPU accelerator + gloo, world 2, against
  torch AdamW over both ranks' batches;
* bench.py's world-8 Ulysses sp8 control flow prints one driver-contract JSON line.
Twin-Flow at world 2 is covered by tests/unit/runtime/test_offload.py (ratio 0.5, ZeRO-3, 2 ranks).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


# ---------------------------------------------------------------------------------------- ZeRO-3 x SP2 x DP2
STEPS, B, S = 3, 2, 32


def _sp_dp_reference():
    """Two data-parallel replicas, each with its own batch; each replica's loss is the mean of the two
    sequence-half losses (what the SP ranks compute); gradients averaged over replicas."""
    model = tiny_llama(num_attention_heads=4, num_key_value_heads=2)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    data = [random_tokens(STEPS, B, S, seed=7 + d) for d in range(2)]
    losses = []
    for s in range(STEPS):
        opt.zero_grad()
        tot = 0.0
        for d in range(2):
            x = data[d][s]
            labels = torch.full_like(x, -100)
            labels[:, :-1] = x[:, 1:]
            logits = model.lm_head(model.model(x))
            per = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), labels.reshape(-1),
                                                    ignore_index=-100, reduction="none").view(B, S)
            valid = (labels != -100).float()
            h = S // 2
            l0 = (per[:, :h] * valid[:, :h]).sum() / valid[:, :h].sum()
            l1 = (per[:, h:] * valid[:, h:]).sum() / valid[:, h:].sum()
            loss = (l0 + l1) / 2 / 2
            loss.backward()
            tot += float(loss)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        losses.append(tot)
    return losses


def _sp_dp_run(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.parallel import groups
    from deepspeedsyclsupport_amd.sequence.layer import enable_sequence_parallel, shard_sequence
    model = tiny_llama(num_attention_heads=4, num_key_value_heads=2)
    cfg = base_config(stage=3, lr=1e-2, mb=B)
    cfg["zero_optimization"]["stage3_param_persistence_threshold"] = 100
    cfg["sequence_parallel"] = {"size": 2}
    cfg["train_batch_size"] = 2 * B  # dp = world / sp = 2
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    assert eng.optimizer.partition and eng.optimizer.coordinator is not None
    # ZeRO partitions over the sequence x data group (all 4 ranks)
    assert eng.optimizer.partition_count() == 4
    sp = groups._get_sequence_parallel_group()
    assert enable_sequence_parallel(eng.module, sp) == 2
    d = dist.get_rank() // 2  # data-parallel replica: ranks {0,1} and {2,3} form the SP groups
    losses = []
    for x in random_tokens(STEPS, B, S, seed=7 + d):
        inp, lab, off = shard_sequence(x, x, sp)
        loss = eng(inp, labels=lab, pos_offset=off, shift_labels=False)
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / 4)
    if dist.get_rank() == 0:
        torch.save(losses, out)


def test_zero3_ulysses_sp2_dp2_world4(tmp_path):
    out = str(tmp_path / "l.pt")
    run_distributed(_sp_dp_run, 4, out)
    got = torch.load(out, weights_only=True)
    ref = _sp_dp_reference()
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-5), (got, ref)


# ---------------------------------------------------------------------------------------- dp8 ZeRO-3 + ZeRO++
def _dp8_reference(steps, mb, seq):
    model = tiny_llama()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01, eps=1e-8)
    data = [random_tokens(steps, mb, seq, seed=300 + r) for r in range(8)]
    losses = []
    for s in range(steps):
        opt.zero_grad()
        tot = 0.0
        for r in range(8):
            loss = model(data[r][s], labels=data[r][s]) / 8
            loss.backward()
            tot += float(loss)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        losses.append(tot)
    return losses


def _dp8_run(zpp, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    rank = dist.get_rank()
    cfg = base_config(stage=3, lr=1e-2, mb=2, clip=1.0)
    cfg["zero_optimization"].update({"stage3_param_persistence_threshold": 0, "stage3_prefetch_bucket_size": 20000,
                                     "stage3_max_live_parameters": 60000, **zpp})
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    coord = eng.optimizer.coordinator
    assert eng.optimizer.partition_count() == 8 and coord is not None
    losses = []
    for x in random_tokens(3, 2, 16, seed=300 + rank):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / 8)
    # the trace recorded on step 1 drives prefetch afterwards
    assert getattr(coord, "trace_complete", True)
    if rank == 0:
        torch.save(losses, out)


@pytest.mark.parametrize("zpp,tol", [({}, 1e-4), ({"zero_hpz_partition_size": 4}, 1e-4),
                                     ({"zero_quantized_weights": True, "zero_hpz_partition_size": 2}, 3e-2)],
                         ids=["plain", "hpz4", "qwz_hpz2"])
def test_dp8_zero3_prefetch_zeropp_world8(zpp, tol, tmp_path):
    out = str(tmp_path / "l.pt")
    run_distributed(_dp8_run, 8, zpp, out)
    got = torch.load(out, weights_only=True)
    ref = _dp8_reference(3, 2, 16)
    assert got == pytest.approx(ref, rel=tol, abs=tol), (got, ref)


# ---------------------------------------------------------------------------------------- BASELINE config 1
def _gpt2_small():
    from transformers import GPT2Config, GPT2LMHeadModel
    torch.manual_seed(0)
    cfg = GPT2Config(n_positions=128, attn_pdrop=0.0, embd_pdrop=0.0, resid_pdrop=0.0)  # GPT-2 small: 124M
    return GPT2LMHeadModel(cfg)


def _gpt2_data(rank, steps=2):
    g = torch.Generator().manual_seed(500 + rank)
    return [torch.randint(0, 50257, (1, 32), generator=g) for _ in range(steps)]


def _gpt2_run(out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    rank = dist.get_rank()
    model = _gpt2_small()
    assert 120e6 < sum(p.numel() for p in model.parameters()) < 130e6
    cfg = {"train_micro_batch_size_per_gpu": 1, "gradient_clipping": 1.0, "steps_per_print": 1000,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "weight_decay": 0.01}},
           "zero_optimization": {"stage": 1, "reduce_bucket_size": int(2e7)}}
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    assert eng.device.type == "cpu" and eng.optimizer.partition_count() == 2
    losses = []
    for x in _gpt2_data(rank):
        loss = eng(input_ids=x, labels=x).loss
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / 2)
    if rank == 0:
        torch.save(losses, out)


def test_baseline_config1_gpt2_small_zero1_gloo_world2(tmp_path):
    out = str(tmp_path / "l.pt")
    run_distributed(_gpt2_run, 2, out)
    got = torch.load(out, weights_only=True)
    model = _gpt2_small()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
    d = [_gpt2_data(0), _gpt2_data(1)]
    ref = []
    for s in range(2):
        opt.zero_grad()
        tot = 0.0
        for r in range(2):
            loss = model(input_ids=d[r][s], labels=d[r][s]).loss / 2
            loss.backward()
            tot += float(loss)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        ref.append(tot)
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-4), (got, ref)


# ---------------------------------------------------------------------------------------- bench.py at world 8
def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_world8_sp8_dryrun():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "8", "--steps", "1", "--warmup", "1",
           "--host-dryrun", "--sp", "8"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp1-sp8"
    assert rec["value"] > 0 and rec["final_loss"] == rec["final_loss"]
