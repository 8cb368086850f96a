"""Elastic training batch-size solver (reference `elasticity/elasticity.py:83-380`, same results for the same config).

Given `max_train_batch_size` and the acceptable `micro_batch_sizes`, choose a global batch size that stays valid for
as many GPU counts as possible: candidates are each micro-batch (and their LCM) scaled by the largest highly
composite number that keeps the batch under the cap (HCNs have the most divisors), and the candidate with the most
valid data-parallel sizes in [min_gpus, max_gpus] wins (ties -> larger or smaller batch per `prefer_larger_batch`).
v0.2 works at node granularity with model parallelism and also returns the micro-batch for the current world size.
"""
import json
import math
import os
from functools import reduce

from .config import (ElasticityConfig, ElasticityConfigError, ElasticityError, ElasticityIncompatibleWorldSize,
                     DEEPSPEED_ELASTICITY_CONFIG, ELASTICITY, LATEST_ELASTICITY_VERSION, MINIMUM_DEEPSPEED_VERSION)
from ..utils.logging import logger

# highly composite numbers (OEIS A002182) up to 720720
HCN_LIST = [1, 2, 4, 6, 12, 24, 36, 48, 60, 120, 180, 240, 360, 720, 840, 1260, 1680, 2520, 5040, 7560, 10080, 15120,
            20160, 25200, 27720, 45360, 50400, 55440, 83160, 110880, 166320, 221760, 277200, 332640, 498960, 554400,
            665280, 720720]


def _largest_hcn_at_most(v):
    best = HCN_LIST[0]
    for h in HCN_LIST:
        if h <= v:
            best = h
        else:
            break
    return best


def get_candidate_batch_sizes(base_list, max_acceptable_batch_size):
    out = set()
    for base in base_list:
        if base >= max_acceptable_batch_size:
            out.add(base)
        else:
            out.add(_largest_hcn_at_most(max_acceptable_batch_size // base) * base)
    return sorted(out)


def get_valid_gpus(batch_size, micro_batches, min_valid_gpus, max_valid_gpus):
    """Every GPU count g in range such that batch_size = mb * k * g for some listed micro-batch mb, k >= 1."""
    valid = set()
    for mb in micro_batches:
        if batch_size % mb:
            continue
        top = batch_size // mb
        for g in range(max(min_valid_gpus, 1), min(top, max_valid_gpus) + 1):
            if top % g == 0:
                valid.add(g)
    return sorted(valid)


def get_best_candidates(candidate_batch_sizes, micro_batches, min_gpus, max_gpus, prefer_larger):
    best_bs, best_gpus = int(min(micro_batches)), None
    best_n = 0
    for bs in candidate_batch_sizes:
        gpus = get_valid_gpus(bs, micro_batches, min_gpus, max_gpus)
        better_tie = (prefer_larger and bs > best_bs) or (not prefer_larger and bs < best_bs)
        if len(gpus) > best_n or (len(gpus) == best_n and better_tie):
            best_n, best_gpus, best_bs = len(gpus), gpus, bs
    return best_bs, best_gpus


def _get_compatible_gpus_v01(micro_batches, max_acceptable_batch_size, min_gpus=None, max_gpus=None,
                             prefer_larger=True):
    min_gpus = min_gpus or 1
    max_gpus = max_gpus or max_acceptable_batch_size // min(micro_batches)
    if any(mb > max_acceptable_batch_size for mb in micro_batches):
        raise ValueError(f"All micro batches must be <= max_acceptable_batch_size {max_acceptable_batch_size}")
    lcm = reduce(lambda a, b: a * b // math.gcd(a, b), micro_batches)
    cands = get_candidate_batch_sizes(list(micro_batches) + [lcm], max_acceptable_batch_size)
    return get_best_candidates(cands, micro_batches, min_gpus, max_gpus, prefer_larger)


def _pick_microbatch(global_bs, dp, micro_batches, prefer_larger):
    fits = [mb for mb in micro_batches if (global_bs // dp) % mb == 0]
    if not fits:
        return None
    return max(fits) if prefer_larger else fits[0]


def _get_compatible_gpus_v02(micro_batches, max_acceptable_batch_size, current_num_gpus, min_gpus=None,
                             max_gpus=None, prefer_larger=True, num_gpus_per_node=1, model_parallel_size=1):
    if num_gpus_per_node % model_parallel_size:
        raise ElasticityError(f"num_gpus_per_node {num_gpus_per_node} must be divisible by model parallel size "
                              f"{model_parallel_size}")
    dp_per_node = num_gpus_per_node // model_parallel_size
    # solve at node granularity, then scale back to data-parallel ranks
    bs, valid_nodes = _get_compatible_gpus_v01(micro_batches, int(max_acceptable_batch_size / dp_per_node),
                                               int(min_gpus / num_gpus_per_node), int(max_gpus / num_gpus_per_node),
                                               prefer_larger=prefer_larger)
    bs = int(bs) * dp_per_node
    valid_dp = [n * dp_per_node for n in valid_nodes]
    if current_num_gpus // model_parallel_size in valid_dp:
        return bs, valid_dp, _pick_microbatch(bs, current_num_gpus, micro_batches, prefer_larger)
    # current size not in the elastic set: best batch for exactly this size
    cur_dp = (current_num_gpus / num_gpus_per_node) * dp_per_node
    cands = [math.floor(max_acceptable_batch_size / float(mb * cur_dp)) * mb * cur_dp for mb in micro_batches]
    bs = max(cands) if prefer_larger else min(cands)
    return bs, [int(cur_dp)], _pick_microbatch(bs, current_num_gpus, micro_batches, prefer_larger)


def _version_tuple(v):
    return tuple(int(x) for x in str(v).split("+")[0].split(".")[:3] if x.isdigit())


def elasticity_enabled(ds_config: dict):
    return bool(ds_config.get(ELASTICITY, {}).get("enabled", False))


def ensure_immutable_elastic_config(runtime_elastic_config_dict: dict):
    if DEEPSPEED_ELASTICITY_CONFIG not in os.environ:
        logger.warning("DEEPSPEED_ELASTICITY_CONFIG not set: cannot verify the scheduler used the same elastic config")
        return
    sched = ElasticityConfig(json.loads(os.environ[DEEPSPEED_ELASTICITY_CONFIG]))
    run = ElasticityConfig(runtime_elastic_config_dict)
    for field in ("max_acceptable_batch_size", "micro_batches", "version"):
        if getattr(sched, field) != getattr(run, field):
            raise ElasticityConfigError(f"Elastic config '{field}' seen by the scheduler ({getattr(sched, field)}) "
                                        f"differs from the runtime's ({getattr(run, field)})")


def compute_elastic_config(ds_config: dict, target_deepspeed_version: str, world_size=0, return_microbatch=False):
    """Returns (final_batch_size, valid_gpus[, micro_batch_size])."""
    if not isinstance(ds_config, dict):
        raise ValueError(f"Expected ds_config to be a dictionary, got {type(ds_config)}")
    if ELASTICITY not in ds_config:
        raise ElasticityConfigError(f"'{ELASTICITY}' is missing from config json")
    ecd = ds_config[ELASTICITY]
    if not ecd.get("enabled", False):
        raise ElasticityConfigError("Elasticity is disabled, set 'enabled': true")
    ec = ElasticityConfig(ecd)
    ver = float(ec.version)
    if ec.model_parallel_size > 1 and ver != 0.2:
        raise ElasticityConfigError(f"Elasticity v{ec.version} does not support model parallelism")
    if ver > LATEST_ELASTICITY_VERSION:
        raise ElasticityConfigError(f"Elasticity version {ec.version} > supported {LATEST_ELASTICITY_VERSION}")
    if _version_tuple(target_deepspeed_version) < _version_tuple(MINIMUM_DEEPSPEED_VERSION):
        raise ElasticityError(f"Target version {target_deepspeed_version} older than {MINIMUM_DEEPSPEED_VERSION}")
    micro = None
    if ver == 0.1:
        bs, valid = _get_compatible_gpus_v01(ec.micro_batches, ec.max_acceptable_batch_size, ec.min_gpus, ec.max_gpus,
                                             ec.prefer_larger_batch_size)
    elif ver == 0.2:
        cur = world_size
        if cur == 0:
            env = os.getenv("WORLD_SIZE", "")
            if not env.isnumeric():
                raise ElasticityConfigError("Elasticity v0.2 needs WORLD_SIZE (argument or environment)")
            cur = int(env)
        bs, valid, micro = _get_compatible_gpus_v02(ec.micro_batches, ec.max_acceptable_batch_size, cur, ec.min_gpus,
                                                    ec.max_gpus, ec.prefer_larger_batch_size, ec.num_gpus_per_node,
                                                    ec.model_parallel_size)
    else:
        raise NotImplementedError(f"Unknown elasticity version {ec.version}")
    bs = int(bs)
    if world_size > 0:
        if world_size not in valid:
            raise ElasticityIncompatibleWorldSize(f"World size {world_size} not in valid GPU counts {valid}")
        mb = next((m for m in sorted(set(ec.micro_batches), reverse=True) if (bs // world_size) % m == 0), None)
        assert mb is not None, f"no micro batch divides {bs} / {world_size}"
        return bs, valid, mb
    if return_microbatch:
        if ver == 0.2:
            return bs, valid, micro
        mb = next((m for m in sorted(set(ec.micro_batches), reverse=True) if bs % m == 0), None)
        return bs, valid, mb
    return bs, valid
