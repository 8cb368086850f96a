"""Native host optimizers vs torch (reference `tests/unit/ops/adam/test_cpu_adam.py`, `ops/adagrad/test_cpu_adagrad.py`,
`ops/lion/test_cpu_lion.py`) and the async tensor I/O handle (reference `tests/unit/ops/aio/test_aio.py`)."""
import pytest
import torch


def _pair(n, seed=0):
    torch.manual_seed(seed)
    a = torch.nn.Parameter(torch.randn(n))
    b = torch.nn.Parameter(a.detach().clone())
    return a, b


def _run(opt_a, opt_b, a, b, steps=5, seed=1):
    g = torch.Generator().manual_seed(seed)
    for _ in range(steps):
        grad = torch.randn(a.shape, generator=g)
        a.grad, b.grad = grad.clone(), grad.clone()
        opt_a.step()
        opt_b.step()


@pytest.mark.parametrize("n", [7, 1024, 65536 + 13])
@pytest.mark.parametrize("adamw", [True, False])
@pytest.mark.parametrize("wd", [0.0, 0.05])
def test_cpu_adam_matches_torch(n, adamw, wd):
    from deepspeedsyclsupport_amd.ops.adam import DeepSpeedCPUAdam
    a, b = _pair(n)
    ours = DeepSpeedCPUAdam([a], lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=wd, adamw_mode=adamw)
    ref_cls = torch.optim.AdamW if adamw else torch.optim.Adam
    ref = ref_cls([b], lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=wd)
    _run(ours, ref, a, b)
    torch.testing.assert_close(a.data, b.data, rtol=1e-5, atol=1e-6)


def test_cpu_adam_writes_low_precision_copy():
    from deepspeedsyclsupport_amd.ops.adam import DeepSpeedCPUAdam
    a, _ = _pair(4096)
    lp = torch.empty(4096, dtype=torch.bfloat16)
    opt = DeepSpeedCPUAdam([a], lr=1e-2)
    a.grad = torch.randn(4096)
    opt.step(fp16_param_groups=[[lp]])
    torch.testing.assert_close(lp, a.data.to(torch.bfloat16), rtol=0, atol=0)


def test_cpu_adagrad_matches_torch():
    from deepspeedsyclsupport_amd.ops.adagrad import DeepSpeedCPUAdagrad
    a, b = _pair(3000)
    ours = DeepSpeedCPUAdagrad([a], lr=1e-2, eps=1e-10, weight_decay=0.01)
    ref = torch.optim.Adagrad([b], lr=1e-2, eps=1e-10, weight_decay=0.01)
    _run(ours, ref, a, b)
    torch.testing.assert_close(a.data, b.data, rtol=1e-5, atol=1e-6)


def test_cpu_lion_matches_reference_rule():
    from deepspeedsyclsupport_amd.ops.lion import DeepSpeedCPULion
    a, b = _pair(2049)
    ours = DeepSpeedCPULion([a], lr=1e-3, betas=(0.9, 0.99), weight_decay=0.1)
    m = torch.zeros_like(b)
    g = torch.Generator().manual_seed(1)
    for _ in range(5):
        grad = torch.randn(a.shape, generator=g)
        a.grad = grad.clone()
        ours.step()
        with torch.no_grad():  # Lion: sign(beta1 m + (1-beta1) g), decoupled decay, m <- beta2 m + (1-beta2) g
            upd = torch.sign(0.9 * m + 0.1 * grad)
            b.mul_(1 - 1e-3 * 0.1).add_(upd, alpha=-1e-3)
            m.mul_(0.99).add_(grad, alpha=0.01)
    torch.testing.assert_close(a.data, b.data, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("use_async", [False, True])
def test_aio_handle_roundtrip(tmp_path, use_async):
    from deepspeedsyclsupport_amd.ops.aio import aio_handle
    h = aio_handle(block_size=1 << 16, queue_depth=8, single_submit=False, overlap_events=True, thread_count=2)
    n = (1 << 20) + 4096
    src = h.new_cpu_locked_tensor(n, torch.empty(0, dtype=torch.uint8))
    src.copy_(torch.randint(0, 255, (n, ), dtype=torch.uint8))
    f = str(tmp_path / "blob.bin")
    if use_async:
        h.async_pwrite(src, f)
        assert h.wait() >= 1
    else:
        h.sync_pwrite(src, f)
    dst = torch.zeros(n, dtype=torch.uint8)
    if use_async:
        h.async_pread(dst, f)
        h.wait()
    else:
        h.sync_pread(dst, f)
    assert torch.equal(dst, src)
    h.free_cpu_locked_tensor(src)
