"""`zero_optimization` config (reference `runtime/zero/config.py:82-317`), same keys and `stage3_*` aliases.

MI355X-first defaults differ where the hardware says so (documented per field): buckets are sized for RCCL over
7 xGMI links and 288 GB of HBM — large enough that each of the 7 peer transfers of a reduce-scatter moves tens
of MB, small enough to keep ≥2 buckets in flight behind backward compute.
"""
import sys
from enum import IntEnum
from typing import Optional

from pydantic import Field, model_validator

from ..config_utils import DeepSpeedConfigModel
from .offload_config import DeepSpeedZeroOffloadOptimizerConfig, DeepSpeedZeroOffloadParamConfig, OffloadDeviceEnum

ZERO_OPTIMIZATION = "zero_optimization"


class ZeroStageEnum(IntEnum):
    disabled = 0
    optimizer_states = 1
    gradients = 2
    weights = 3
    max_stage = 3


class DeepSpeedZeroConfig(DeepSpeedConfigModel):
    stage: ZeroStageEnum = 0
    contiguous_gradients: bool = True
    reduce_scatter: bool = True
    reduce_bucket_size: int = Field(int(5e8), ge=0)
    use_multi_rank_bucket_allreduce: bool = True
    allgather_partitions: bool = True
    allgather_bucket_size: int = Field(int(5e8), ge=0)
    overlap_comm: Optional[bool] = None
    load_from_fp32_weights: bool = True
    elastic_checkpoint: bool = False
    offload_param: Optional[DeepSpeedZeroOffloadParamConfig] = None
    offload_optimizer: Optional[DeepSpeedZeroOffloadOptimizerConfig] = None
    sub_group_size: int = Field(int(1e9), ge=0)
    cpu_offload_param: Optional[bool] = None
    cpu_offload_use_pin_memory: Optional[bool] = None
    cpu_offload: Optional[bool] = None
    prefetch_bucket_size: int = Field(int(5e7), ge=0, alias="stage3_prefetch_bucket_size")
    param_persistence_threshold: int = Field(int(1e5), ge=0, alias="stage3_param_persistence_threshold")
    model_persistence_threshold: int = Field(sys.maxsize, ge=0, alias="stage3_model_persistence_threshold")
    max_live_parameters: int = Field(int(1e9), ge=0, alias="stage3_max_live_parameters")
    max_reuse_distance: int = Field(int(1e9), ge=0, alias="stage3_max_reuse_distance")
    gather_16bit_weights_on_model_save: bool = Field(False, alias="stage3_gather_16bit_weights_on_model_save")
    stage3_gather_fp16_weights_on_model_save: bool = False
    ignore_unused_parameters: bool = True
    legacy_stage1: bool = False
    grad_hooks: bool = True
    round_robin_gradients: bool = False
    zero_hpz_partition_size: int = Field(1, ge=0)
    zero_quantized_weights: bool = False
    zero_quantized_nontrainable_weights: bool = False
    zero_quantized_gradients: bool = False
    mics_shard_size: int = -1
    mics_hierarchical_params_gather: bool = False
    memory_efficient_linear: bool = True
    pipeline_loading_checkpoint: bool = False
    override_module_apply: bool = True
    # debug mode: cross-rank consistency check before every ZeRO collective (runtime/zero/utils.py)
    safe_mode: bool = False
    # MoE expert-parameter gradient averaging: "global" = mean over the whole data-parallel batch (dense DP size, the
    # default here); "expert_dp" = mean over the expert-data-parallel group only, i.e. ep_size times larger — the
    # reference's `stage_1_and_2.py average_tensor` / `engine._reduce_expert_gradients` numerics.
    moe_expert_grad_scaling: str = "global"

    @model_validator(mode="after")
    def _fixups(self):
        # legacy boolean offload flags -> structured sub-configs (reference validators)
        if self.cpu_offload and self.offload_optimizer is None:
            object.__setattr__(self, "offload_optimizer",
                               DeepSpeedZeroOffloadOptimizerConfig(device=OffloadDeviceEnum.cpu,
                                                                   pin_memory=bool(self.cpu_offload_use_pin_memory)))
        if self.cpu_offload_param and self.offload_param is None:
            object.__setattr__(self, "offload_param",
                               DeepSpeedZeroOffloadParamConfig(device=OffloadDeviceEnum.cpu,
                                                               pin_memory=bool(self.cpu_offload_use_pin_memory)))
        if self.stage3_gather_fp16_weights_on_model_save:
            object.__setattr__(self, "gather_16bit_weights_on_model_save", True)
        if self.overlap_comm is None:
            object.__setattr__(self, "overlap_comm", self.stage == ZeroStageEnum.weights)
        return self

    @property
    def offload_optimizer_device(self):
        return self.offload_optimizer.device if self.offload_optimizer else OffloadDeviceEnum.none

    @property
    def offload_param_device(self):
        return self.offload_param.device if self.offload_param else OffloadDeviceEnum.none


def read_zero_config_deprecated(param_dict):
    zero = {}
    zero["stage"] = 1 if param_dict[ZERO_OPTIMIZATION] else 0
    if zero["stage"] > 0:
        zero["allgather_bucket_size"] = param_dict.get("allgather_size", int(5e8))
    return zero


def get_zero_config(param_dict):
    if ZERO_OPTIMIZATION in param_dict:
        zero = param_dict[ZERO_OPTIMIZATION]
        if isinstance(zero, bool):
            zero = read_zero_config_deprecated(param_dict)
    else:
        zero = {}
    return DeepSpeedZeroConfig(**zero)
