"""Comm facade API parity (reference `tests/unit/comm/test_dist.py`): coalesced all-gather, env discovery for MPI,
AzureML and SageMaker launchers."""
import os

import pytest
import torch

from ..common import run_distributed


def _coalesced(out):
    from deepspeedsyclsupport_amd import comm as dist
    r, w = dist.get_rank(), dist.get_world_size()
    ins = [torch.full((3, ), float(r)), torch.full((5, ), 10.0 + r)]
    outs = [torch.empty(3 * w), torch.empty(5 * w)]
    dist.all_gather_coalesced(outs, ins)
    t = torch.tensor([1.0 + r])
    dist.all_reduce_coalesced([t])
    if r == 0:
        torch.save({"outs": outs, "sum": t}, out)


def test_all_gather_coalesced(tmp_path):
    out = str(tmp_path / "c.pt")
    run_distributed(_coalesced, 2, out)
    d = torch.load(out, weights_only=True)
    torch.testing.assert_close(d["outs"][0], torch.tensor([0., 0, 0, 1, 1, 1]))
    torch.testing.assert_close(d["outs"][1], torch.tensor([10.] * 5 + [11.] * 5))
    assert float(d["sum"]) == 3.0


@pytest.fixture
def clean_env(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def test_env_discovery(clean_env):
    from deepspeedsyclsupport_amd import comm as dist
    clean_env.setenv("OMPI_COMM_WORLD_RANK", "3")
    clean_env.setenv("OMPI_COMM_WORLD_SIZE", "8")
    clean_env.setenv("OMPI_COMM_WORLD_LOCAL_RANK", "3")
    dist.mpi_discovery(distributed_port=29511, verbose=False)
    assert (os.environ["RANK"], os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"]) == ("3", "8", "3")
    assert os.environ["MASTER_PORT"] == "29511"
    clean_env.setenv("OMPI_COMM_WORLD_LOCAL_SIZE", "4")
    clean_env.setenv("AZ_BATCH_MASTER_NODE", "10.0.0.7:6000")
    clean_env.setenv("AZUREML_EXPERIMENT_ID", "x")
    clean_env.delenv("MASTER_PORT", raising=False)
    assert dist.in_aml() and not dist.in_aws_sm()
    dist.patch_aml_env_for_torch_nccl_backend(master_port=6105, verbose=False)
    assert os.environ["MASTER_ADDR"] == "10.0.0.7" and os.environ["MASTER_PORT"] == "6105"
    clean_env.setenv("SM_TRAINING_ENV", "{}")
    dist.patch_aws_sm_env_for_torch_nccl_backend(verbose=False)
    assert os.environ["RANK"] == "3"
