"""Elastic batch-size solver (reference `tests/unit/elasticity/test_elastic.py`; expected values are the
reference's published test expectations for the same configs)."""
import os

import pytest

from deepspeedsyclsupport_amd import __version__ as ds_version
from deepspeedsyclsupport_amd import elasticity
from deepspeedsyclsupport_amd.elasticity.config import ElasticityError, ElasticityIncompatibleWorldSize


@pytest.fixture
def ds_config():
    return {"elasticity": {"enabled": True, "max_train_batch_size": 10000, "micro_batch_sizes": [8, 12, 16, 17],
                           "min_gpus": 32, "max_gpus": 1500, "min_time": 20, "version": 0.1}}


def test_basic_10k(ds_config):
    bs, valid = elasticity.compute_elastic_config(ds_config, ds_version)
    for g in valid:
        assert bs % g == 0 and any((bs // g) % mb == 0 for mb in ds_config["elasticity"]["micro_batch_sizes"])
    assert len(valid) == 23
    assert bs == 9792


def test_old_version(ds_config):
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, "0.2")


def test_disabled(ds_config):
    ds_config["elasticity"]["enabled"] = False
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, ds_version)


def test_valid_world_size(ds_config):
    _, _, mb = elasticity.compute_elastic_config(ds_config, ds_version, world_size=64)
    assert mb == 17


def test_invalid_world_size(ds_config):
    with pytest.raises(ElasticityIncompatibleWorldSize):
        elasticity.compute_elastic_config(ds_config, ds_version, world_size=128)


def test_future_version(ds_config):
    ds_config["elasticity"]["version"] = "0.3"
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, ds_version)


@pytest.mark.parametrize("missing", ["max_train_batch_size", "micro_batch_sizes"])
def test_missing_keys(ds_config, missing):
    del ds_config["elasticity"][missing]
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, ds_version)


def test_model_parallel(ds_config):
    ds_config["elasticity"].update(model_parallel_size=4, num_gpus_per_node=8, version=0.1)
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, ds_version)
    ds_config["elasticity"].update(model_parallel_size=16, version=0.2)
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, ds_version, world_size=16)
    ds_config["elasticity"].update(model_parallel_size=4)
    os.environ["WORLD_SIZE"] = "16"
    try:
        elasticity.compute_elastic_config(ds_config, ds_version)
    finally:
        os.environ.pop("WORLD_SIZE")


@pytest.mark.parametrize("key,value", [("micro_batch_sizes", [1, 4, -1, 2, -10]), ("min_gpus", -1), ("max_gpus", -1),
                                       ("micro_batch_sizes", 5), ("micro_batch_sizes", ["a", None, 0.5]),
                                       ("micro_batch_sizes", [2, 0.5, 4])])
def test_invalid_values(ds_config, key, value):
    ds_config["elasticity"][key] = value
    with pytest.raises(ElasticityError):
        elasticity.compute_elastic_config(ds_config, ds_version)


def test_proper_mbsz(ds_config):
    ds_config["elasticity"].update(max_train_batch_size=32, micro_batch_sizes=[1, 2, 3, 7], min_gpus=1)
    _, _, mb = elasticity.compute_elastic_config(ds_config, ds_version, world_size=7)
    assert mb == 3


def test_engine_config_override():
    from deepspeedsyclsupport_amd.runtime.config import DeepSpeedConfig
    cfg = {"elasticity": {"enabled": True, "max_train_batch_size": 96, "micro_batch_sizes": [2, 4],
                          "min_gpus": 1, "max_gpus": 8, "version": 0.1}, "optimizer": {"type": "Adam"}}
    c = DeepSpeedConfig(cfg, world_size=4)
    assert c.train_batch_size == c.train_micro_batch_size_per_gpu * c.gradient_accumulation_steps * 4
    bad = dict(cfg, train_batch_size=10)
    with pytest.raises(ElasticityError):
        DeepSpeedConfig(bad, world_size=4)
