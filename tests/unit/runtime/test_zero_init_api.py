"""zero.Init per-parameter API (`p.all_gather()` / `p.partition()`, `ds_*` attributes), init-context suspension in
`initialize()`, and `register_external_parameter` under ZeRO-3 (reference `partition_parameters.py:1336-1338`,
register_external_parameter; `tests/unit/runtime/zero/test_zero_context*.py`)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..common import run_distributed


def _per_param_api():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    torch.manual_seed(dist.get_rank())  # rank-dependent init: Init must broadcast rank 0's values
    with ds.zero.Init():
        lin = nn.Linear(10, 7)
    w = lin.weight
    assert w.numel() == 0 and w.ds_numel == 70 and tuple(w.ds_shape) == (7, 10)
    w.all_gather()
    assert tuple(w.shape) == (7, 10)
    full = w.data.clone()
    ref = full.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(full, ref)  # identical on every rank
    w.partition()
    assert w.numel() == 0
    # both params at once through param_list
    w.all_gather(param_list=[lin.weight, lin.bias])
    assert lin.bias.shape == (7, )
    w.partition(param_list=[lin.weight, lin.bias])
    assert lin.bias.numel() == 0


def test_per_param_all_gather_partition():
    run_distributed(_per_param_api, 2)


V, H = 32, 16


class Head(nn.Module):
    """LM head tied to the embedding, which it does NOT own (kept out of its module tree)."""

    def __init__(self, emb):
        super().__init__()
        self.__dict__["emb"] = emb

    def forward(self, h):
        return F.linear(h, self.emb.weight)


class Tied(nn.Module):

    def __init__(self):
        super().__init__()
        self.embed = nn.Embedding(V, H)
        self.body = nn.Linear(H, H)
        self.head = Head(self.embed)

    def forward(self, x, labels=None):
        logits = self.head(torch.tanh(self.body(self.embed(x))))
        return F.cross_entropy(logits.reshape(-1, V).float(), labels.reshape(-1))


def _tied_run(register, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    torch.manual_seed(0)
    model = Tied()
    if register:
        ds.zero.register_external_parameter(model.head, model.embed.weight)
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0}}
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    assert eng.optimizer.partition_count() == 2
    losses = []
    g = torch.Generator().manual_seed(5 + dist.get_rank())
    for _ in range(3):
        x = torch.randint(0, V, (2, 6), generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(float(t) / 2)
    if dist.get_rank() == 0:
        torch.save(losses, out)


def test_register_external_parameter_zero3(tmp_path):
    out = str(tmp_path / "l.pt")
    run_distributed(_tied_run, 2, True, out)
    got = torch.load(out, weights_only=True)
    torch.manual_seed(0)
    model = Tied()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.0)  # the engine's AdamW default
    gens = [torch.Generator().manual_seed(5 + r) for r in range(2)]
    ref = []
    for _ in range(3):
        opt.zero_grad()
        tot = 0.0
        for r in range(2):
            x = torch.randint(0, V, (2, 6), generator=gens[r])
            loss = model(x, labels=x) / 2
            loss.backward()
            tot += float(loss)
        opt.step()
        ref.append(tot)
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-5), (got, ref)


def test_unregistered_external_parameter_fails(tmp_path):
    """Without the registration the head sees the embedding's empty partition placeholder."""
    with pytest.raises(AssertionError):
        run_distributed(_tied_run, 2, False, str(tmp_path / "l.pt"))
