"""Activation checkpointing (reference `tests/unit/runtime/activation_checkpointing/test_activation_checkpointing.py`:
checkpointed vs plain forward/backward must give the same outputs and gradients, for tensor / non-tensor / multi-output
segments, with partitioned, contiguous and host-resident checkpoints, reentrant and non-reentrant)."""
import pytest
import torch
import torch.nn as nn

from ...common import run_distributed


def _ckpt():
    from deepspeedsyclsupport_amd.runtime.activation_checkpointing import checkpointing
    return checkpointing


class _Block(nn.Module):

    def __init__(self, h=32, p=0.1):
        super().__init__()
        self.a, self.b = nn.Linear(h, 2 * h), nn.Linear(2 * h, h)
        self.drop = nn.Dropout(p)

    def forward(self, x, scale=1.0, mask=None):
        y = self.b(self.drop(torch.relu(self.a(x)))) * scale
        if mask is not None:
            y = y.masked_fill(mask, 0.0)
        return x + y


def _run(blocks, x, how, mask=None):
    ck = _ckpt()
    h = x
    for blk in blocks:
        if how == "plain":
            h = blk(h, 0.5, mask)
        elif how == "reentrant":
            h = ck.checkpoint(blk, h, 0.5, mask)
        else:
            h = ck.non_reentrant_checkpoint(blk, h, 0.5, mask)
    return h


def _grads(blocks, x, how, mask=None, seed=3):
    torch.manual_seed(seed)
    for b in blocks:
        b.zero_grad()
    xx = x.clone().requires_grad_(True)
    out = _run(blocks, xx, how, mask)
    out.pow(2).mean().backward()
    return out.detach(), xx.grad.clone(), [p.grad.clone() for b in blocks for p in b.parameters()]


@pytest.mark.parametrize("how", ["reentrant", "non_reentrant"])
@pytest.mark.parametrize("with_mask", [False, True])
def test_checkpoint_matches_plain_with_dropout_replay(how, with_mask):
    ck = _ckpt()
    ck.configure(None, partition_activations=False, contiguous_checkpointing=False, checkpoint_in_cpu=False)
    torch.manual_seed(0)
    blocks = nn.ModuleList([_Block() for _ in range(3)])
    x = torch.randn(4, 6, 32)
    mask = (torch.rand(4, 6, 1) > 0.8) if with_mask else None
    o0, gx0, gp0 = _grads(blocks, x, "plain", mask)
    o1, gx1, gp1 = _grads(blocks, x, how, mask)
    torch.testing.assert_close(o1, o0, rtol=0, atol=0)
    torch.testing.assert_close(gx1, gx0, rtol=1e-6, atol=1e-7)
    for a, b in zip(gp1, gp0):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_multiple_outputs_and_non_float_outputs():
    ck = _ckpt()
    ck.configure(None, partition_activations=False, contiguous_checkpointing=False, checkpoint_in_cpu=False)
    lin = nn.Linear(8, 8)

    def seg(x):
        y = lin(x)
        return y, (y > 0), y.sum(-1)

    x = torch.randn(3, 8, requires_grad=True)
    y, m, s = ck.checkpoint(seg, x)
    assert m.dtype == torch.bool and not m.requires_grad
    (y.sum() + s.sum()).backward()
    g = x.grad.clone()
    x.grad = None
    y2, _, s2 = seg(x)
    (y2.sum() + s2.sum()).backward()
    torch.testing.assert_close(g, x.grad)


class _FakeMPU:

    def __init__(self, group, rank, size):
        self.g, self.r, self.s = group, rank, size

    def get_model_parallel_rank(self):
        return self.r

    def get_model_parallel_world_size(self):
        return self.s

    def get_model_parallel_group(self):
        return self.g


def _partitioned(how, contiguous):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    ds.init_distributed(dist_backend="gloo")
    ck = _ckpt()
    mpu = _FakeMPU(None, dist.get_rank(), dist.get_world_size())
    torch.manual_seed(0)  # same weights and inputs on both "tensor-parallel" ranks (replicated activations)
    blocks = nn.ModuleList([_Block() for _ in range(4)])
    x = torch.randn(4, 6, 32)
    ck.configure(None, partition_activations=False, contiguous_checkpointing=False, checkpoint_in_cpu=False)
    o0, gx0, gp0 = _grads(blocks, x, "plain")
    ck.configure(mpu, partition_activations=True, contiguous_checkpointing=contiguous, num_checkpoints=4,
                 checkpoint_in_cpu=False)
    sizes = []
    orig = ck._Saved.__init__

    def spy(self, t, arg_idx=0):
        orig(self, t, arg_idx)
        sizes.append((t.numel(), self.data.numel(), self.partitioned, self.pooled))

    ck._Saved.__init__ = spy
    try:
        for it in range(3):
            o1, gx1, gp1 = _grads(blocks, x, how)
            torch.testing.assert_close(o1, o0, rtol=0, atol=0)
            torch.testing.assert_close(gx1, gx0, rtol=1e-6, atol=1e-7)
            for a, b in zip(gp1, gp0):
                torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
            if contiguous:
                if it == 0:
                    first = ck._POOL.allocations
                    assert first >= 1
                    # every checkpoint of the iteration sits in one [4, n] buffer, slot after slot
                    (buf, ) = [b for k, b in ck._POOL.buffers.items() if k[1] == x.numel() // 2]
                    assert buf.shape == (4, x.numel() // 2)
                assert ck._POOL.allocations == first, "buffers must be reused across iterations"
                ck.reset()
    finally:
        ck._Saved.__init__ = orig
    big = [s for s in sizes if s[0] == x.numel()]
    assert big and all(kept == full // 2 and part for full, kept, part, _ in big)  # each rank keeps half
    assert all(pooled == contiguous for _, _, _, pooled in big)


@pytest.mark.parametrize("how", ["reentrant", "non_reentrant"])
@pytest.mark.parametrize("contiguous", [False, True])
def test_partitioned_activations_two_ranks(how, contiguous):
    run_distributed(_partitioned, 2, how, contiguous)


def test_contiguous_pool_grows_past_announced_checkpoints():
    ck = _ckpt()
    ck.num_layers = 2
    pool = ck._ContiguousPool()
    slots = [pool.slot(0, 16, torch.float32, "cpu", False) for _ in range(5)]
    for i, s in enumerate(slots):
        s.fill_(float(i))
    assert [float(s[0]) for s in slots] == [0.0, 1.0, 2.0, 3.0, 4.0]  # earlier slots survive the growth
    pool.rewind()
    again = pool.slot(0, 16, torch.float32, "cpu", False)
    assert again.data_ptr() == pool.buffers[(0, 16, torch.float32, "cpu", False)][0].data_ptr()


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["reentrant", "non_reentrant"])
def test_cpu_checkpointing_gpu(how):
    """Checkpoints parked in pinned host memory over the side stream: same gradients, inputs really leave the HBM."""
    ck = _ckpt()
    torch.manual_seed(0)
    blocks = nn.ModuleList([_Block(64, p=0.0) for _ in range(3)]).cuda()
    x = torch.randn(8, 16, 64, device="cuda")
    ck.configure(None, partition_activations=False, contiguous_checkpointing=False, checkpoint_in_cpu=False)
    o0, gx0, gp0 = _grads(blocks, x, "plain")
    ck.configure(None, partition_activations=False, contiguous_checkpointing=False, checkpoint_in_cpu=True)
    seen = []
    orig = ck._Saved.__init__

    def spy(self, t, arg_idx=0):
        orig(self, t, arg_idx)
        seen.append((self.on_host, self.data.is_pinned() if not self.data.is_cuda else False))

    ck._Saved.__init__ = spy
    try:
        o1, gx1, gp1 = _grads(blocks, x, how)
    finally:
        ck._Saved.__init__ = orig
        ck.configure(None, checkpoint_in_cpu=False)
    assert any(h and pinned for h, pinned in seen)
    torch.testing.assert_close(o1, o0, rtol=0, atol=0)
    torch.testing.assert_close(gx1, gx0, rtol=1e-5, atol=1e-6)
    for a, b in zip(gp1, gp0):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
