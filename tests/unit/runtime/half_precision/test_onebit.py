"""1-bit Adam / 0-1 Adam / 1-bit LAMB (reference `tests/unit/runtime/half_precision/onebit/test_onebit.py`) and the
compressed all-reduce (`tests/onebit/test_nccl_backend.py`)."""
import pytest
import torch

from ...common import run_distributed
from ...simple_model import base_config, random_tokens, tiny_llama


def test_pack_unpack_roundtrip():
    from deepspeedsyclsupport_amd.runtime.comm.compressed import pack_signs, unpack_signs
    x = torch.randn(64)
    assert torch.equal(unpack_signs(pack_signs(x)), torch.where(x >= 0, 1.0, -1.0))


def _compressed(out):
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.runtime.comm.compressed import CompressedBackend
    be = CompressedBackend()
    r, W = dist.get_rank(), dist.get_world_size()
    n = 100
    N = be.padded_size(n)
    we, se = torch.zeros(N), torch.zeros(N // W)
    # +-c vectors compress losslessly: the result must be the exact average
    g = torch.Generator().manual_seed(5)
    signs = [torch.where(torch.rand(n, generator=g) > 0.5, 1.0, -1.0) for _ in range(W)]
    x = signs[r] * (r + 1.0)
    y = x.clone()
    be.compressed_allreduce(y, we, se)
    exact = sum(s * (i + 1.0) for i, s in enumerate(signs)) / W
    # error feedback: averaging the compressed results of repeated all-reduces of the same input converges
    acc = torch.zeros(n)
    z_in = torch.randn(n, generator=torch.Generator().manual_seed(10 + r))
    we.zero_(), se.zero_()
    T = 200
    for _ in range(T):
        z = z_in.clone()
        be.compressed_allreduce(z, we, se)
        acc += z
    tz = z_in.clone()
    dist.all_reduce(tz)
    if r == 0:
        torch.save({"y": y, "exact": exact, "avg": acc / T, "true": tz / W}, out)


def test_compressed_allreduce(tmp_path):
    out = str(tmp_path / "c.pt")
    run_distributed(_compressed, 2, out)
    d = torch.load(out, weights_only=True)
    # sign-exact inputs are not lossless (scale is an L2 mean), but the error-feedback time average is unbiased
    err = (d["avg"] - d["true"]).abs()
    assert err.mean() < 0.02 and err.max() < 0.1, (err.mean(), err.max())
    assert torch.sign(d["y"]).eq(torch.sign(d["exact"])).float().mean() > 0.9


def _onebit_run(opt_type, params, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    cfg = base_config(stage=0, lr=1e-2, mb=2, clip=0.0)
    cfg["optimizer"] = {"type": opt_type, "params": dict(lr=2e-3, **params)}
    eng, opt, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    data = random_tokens(8, 2, 16, seed=11 + dist.get_rank())
    losses = []
    for i in range(8):
        x = data[i % 2]  # a repeated pair of batches: the loss must go down
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    # every rank must hold identical parameters (the compressed all-reduce returns the same tensor everywhere)
    flat = torch.cat([p.detach().float().reshape(-1) for p in eng.module.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other), "ranks diverged"
    assert eng.optimizer._local_grads(), "compression stage not reached"
    if dist.get_rank() == 0:
        torch.save({"losses": losses}, out)


@pytest.mark.parametrize("opt_type,params", [("OneBitAdam", {"freeze_step": 3}),
                                             ("ZeroOneAdam", {"var_freeze_step": 3, "var_update_scaler": 2,
                                                              "local_step_clipper": 2}),
                                             ("OneBitLamb", {"freeze_step": 3})])
def test_onebit_optimizers(opt_type, params, tmp_path):
    out = str(tmp_path / "o.pt")
    run_distributed(_onebit_run, 2, opt_type, params, out)
    losses = torch.load(out, weights_only=True)["losses"]
    assert min(losses[-2:]) < losses[0], losses
