"""DeepSpeed JSON config (reference `runtime/config.py:696-1027`): same keys, same batch-triple solve.

Accepts a dict, a path to a JSON/hjson file, or a base64-encoded JSON string. Top-level scalar keys are
exposed as attributes with the reference's names (`train_batch_size`, `fp16_enabled`, `zero_optimization_stage`,
...); structured sections are pydantic models (`zero_config`, `comms_config`, ...).
"""
import base64
import copy
import json
import os
from typing import Optional

import torch
from pydantic import Field

from ..utils.logging import logger
from .config_utils import DeepSpeedConfigModel, ScientificNotationEncoder, dict_raise_error_on_duplicate_keys
from .zero.config import ZeroStageEnum, get_zero_config

ADAM_OPTIMIZER = "adam"
ADAMW_OPTIMIZER = "adamw"
LAMB_OPTIMIZER = "lamb"
ONEBIT_ADAM_OPTIMIZER = "onebitadam"
ZERO_ONE_ADAM_OPTIMIZER = "zerooneadam"
ONEBIT_LAMB_OPTIMIZER = "onebitlamb"
ADAGRAD_OPTIMIZER = "adagrad"
LION_OPTIMIZER = "lion"
MUADAM_OPTIMIZER = "muadam"
MUADAMW_OPTIMIZER = "muadamw"
MUSGD_OPTIMIZER = "musgd"
SGD_OPTIMIZER = "sgd"
DEEPSPEED_OPTIMIZERS = [
    ADAM_OPTIMIZER, ADAMW_OPTIMIZER, LAMB_OPTIMIZER, ONEBIT_ADAM_OPTIMIZER, ONEBIT_LAMB_OPTIMIZER,
    ZERO_ONE_ADAM_OPTIMIZER, ADAGRAD_OPTIMIZER, LION_OPTIMIZER, MUADAM_OPTIMIZER, MUADAMW_OPTIMIZER, MUSGD_OPTIMIZER,
    SGD_OPTIMIZER
]
TORCH_ADAM_PARAM = "torch_adam"
ADAM_W_MODE = "adam_w_mode"
MAX_GRAD_NORM = "max_grad_norm"


class ValidationMode:
    """How checkpoint tag mismatches across ranks are treated (`checkpoint.tag_validation`)."""
    WARN = "WARN"
    IGNORE = "IGNORE"
    FAIL = "FAIL"


class DeepSpeedConfigError(Exception):
    pass


# ------------------------------------------------------------------------------------------- sub-configs
class FP16Config(DeepSpeedConfigModel):
    enabled: bool = False
    auto_cast: bool = False
    loss_scale: float = 0.0
    initial_scale_power: int = 16
    loss_scale_window: int = 1000
    hysteresis: int = 2
    consecutive_hysteresis: bool = False
    min_loss_scale: float = 1.0
    fp16_master_weights_and_grads: bool = False
    type: Optional[str] = None


class BF16Config(DeepSpeedConfigModel):
    enabled: bool = False
    immediate_grad_update: bool = False
    # MI355X addition: keep the fp32 master as (bf16 weight, 16-bit residual) instead of a separate fp32 copy:
    # 2 B/param less optimizer state, bit-exact fp32 master arithmetic (weights rounded half away from zero)
    split_master_weights: bool = False


class AMPConfig(DeepSpeedConfigModel):
    model_config = dict(extra="allow")
    enabled: bool = False


class CommsLoggerConfig(DeepSpeedConfigModel):
    enabled: bool = False
    prof_all: bool = True
    prof_ops: list = []
    verbose: bool = False
    debug: bool = False


class FlopsProfilerConfig(DeepSpeedConfigModel):
    enabled: bool = False
    recompute_fwd_factor: float = 0.0
    profile_step: int = 1
    module_depth: int = -1
    top_modules: int = 1
    detailed: bool = True
    output_file: Optional[str] = None


class ActivationCheckpointingConfig(DeepSpeedConfigModel):
    partition_activations: bool = False
    contiguous_memory_optimization: bool = False
    cpu_checkpointing: bool = False
    number_checkpoints: Optional[int] = None
    synchronize_checkpoint_boundary: bool = False
    profile: bool = False


class TensorBoardConfig(DeepSpeedConfigModel):
    enabled: bool = False
    output_path: str = ""
    job_name: str = "DeepSpeedJobName"


class WandbConfig(DeepSpeedConfigModel):
    enabled: bool = False
    group: Optional[str] = None
    team: Optional[str] = None
    project: str = "deepspeed"


class CSVConfig(DeepSpeedConfigModel):
    enabled: bool = False
    output_path: str = ""
    job_name: str = "DeepSpeedJobName"


class MonitorConfig(DeepSpeedConfigModel):
    tensorboard: TensorBoardConfig = TensorBoardConfig()
    wandb: WandbConfig = WandbConfig()
    csv_monitor: CSVConfig = CSVConfig()

    @property
    def enabled(self):
        return self.tensorboard.enabled or self.wandb.enabled or self.csv_monitor.enabled


class AIOConfig(DeepSpeedConfigModel):
    block_size: int = 1048576
    queue_depth: int = 8
    thread_count: int = 1
    single_submit: bool = False
    overlap_events: bool = True


class CheckpointConfig(DeepSpeedConfigModel):
    tag_validation: str = "Warn"
    load_universal: bool = False
    # also write the optimizer state in the reference's own layout under <save_dir>/reference_format/<tag>
    # (`checkpoint/reference_format.py`), for tools written against the reference's files
    write_reference_format: bool = False
    use_node_local_storage: bool = False
    parallel_write: dict = {}


class DataTypesConfig(DeepSpeedConfigModel):
    grad_accum_dtype: Optional[str] = None


class PipelineConfig(DeepSpeedConfigModel):
    model_config = dict(extra="allow")
    stages: str = "auto"
    partition: str = "best"
    seed_layers: bool = False
    activation_checkpoint_interval: int = 0
    pipe_partitioned: bool = True
    grad_partitioned: bool = True


class HybridEngineConfig(DeepSpeedConfigModel):
    enabled: bool = False
    max_out_tokens: int = 512
    inference_tp_size: int = 1
    release_inference_cache: bool = False
    pin_parameters: bool = True
    tp_gather_partition_size: int = 8


class ElasticityConfigModel(DeepSpeedConfigModel):
    model_config = dict(extra="allow")
    enabled: bool = False


class SequenceParallelConfig(DeepSpeedConfigModel):
    """MI355X addition: Ulysses SP size when no `mpu` is passed (groups built over consecutive ranks)."""
    size: int = Field(1, ge=1)
    communication_data_type: Optional[str] = None


def _dtype_from_str(s):
    if s is None:
        return None
    s = str(s).lower()
    return {"fp32": torch.float32, "float32": torch.float32, "fp16": torch.float16, "float16": torch.float16,
            "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}[s]


class DeepSpeedConfig:
    """Parsed configuration. `world_size` is the data-parallel size used by the batch solve."""

    def __init__(self, config, mpu=None, world_size=None):
        if isinstance(config, dict):
            self._param_dict = copy.deepcopy(config)
        elif isinstance(config, str) and os.path.exists(config):
            with open(config) as f:
                text = f.read()
            try:
                self._param_dict = json.loads(text, object_pairs_hook=dict_raise_error_on_duplicate_keys)
            except json.JSONDecodeError:
                import yaml  # hjson-like leniency through YAML (JSON superset)
                self._param_dict = yaml.safe_load(text)
        elif isinstance(config, str):
            try:
                self._param_dict = json.loads(base64.urlsafe_b64decode(config).decode("utf-8"))
            except Exception as e:
                raise ValueError(f"Expected a path, dict or base64 JSON string as DeepSpeed config, got {config!r}") from e
        else:
            raise ValueError(f"Unsupported config type {type(config)}")

        from .. import comm as dist
        if world_size is not None:
            self.world_size = world_size
        elif mpu is not None:
            self.world_size = mpu.get_data_parallel_world_size()
        else:
            sp = self._param_dict.get("sequence_parallel", {}).get("size", 1)
            self.world_size = max(dist.get_world_size() // sp, 1)
        self.global_rank = dist.get_rank()
        self.elasticity_enabled = self._apply_elasticity(self._param_dict)
        self._initialize_params(self._param_dict)
        self._configure_train_batch_size()
        self._do_sanity_check()

    def _apply_elasticity(self, p):
        """Elastic batch sizing overrides the batch triple (reference `runtime/config.py:723-785`)."""
        from ..elasticity import compute_elastic_config, elasticity_enabled, ensure_immutable_elastic_config
        from ..elasticity.config import ElasticityConfigError
        if not elasticity_enabled(p):
            return False
        from .. import __version__
        ensure_immutable_elastic_config(p["elasticity"])
        mp = p["elasticity"].get("model_parallel_size", 1)
        bs, valid, mb = compute_elastic_config(p, __version__, world_size=self.world_size * 1, return_microbatch=True)
        if mp > 1:
            pass  # world_size above is already data-parallel
        ignore = p["elasticity"].get("ignore_non_elastic_batch_info", False)
        if not ignore:
            for key in ("train_batch_size", "train_micro_batch_size_per_gpu", "gradient_accumulation_steps"):
                if key in p:
                    raise ElasticityConfigError(f"'{key}' must not be set when elasticity is enabled (found "
                                                f"{p[key]}); set 'ignore_non_elastic_batch_info': true to override")
        p["train_batch_size"] = bs
        p["train_micro_batch_size_per_gpu"] = mb
        p["gradient_accumulation_steps"] = bs // (mb * self.world_size)
        self.elastic_valid_gpus = valid
        return True

    # --------------------------------------------------------------------------------------- parse
    def _initialize_params(self, p):
        self.train_batch_size = p.get("train_batch_size")
        self.train_micro_batch_size_per_gpu = p.get("train_micro_batch_size_per_gpu")
        self.gradient_accumulation_steps = p.get("gradient_accumulation_steps")
        self.steps_per_print = p.get("steps_per_print", 10)
        self.dump_state = p.get("dump_state", False)
        self.disable_allgather = p.get("disable_allgather", False)
        self.communication_data_type = _dtype_from_str(p.get("communication_data_type"))
        self.seq_parallel_communication_data_type = _dtype_from_str(
            p.get("seq_parallel_communication_data_type", "fp32"))
        self.prescale_gradients = p.get("prescale_gradients", False)
        self.gradient_predivide_factor = p.get("gradient_predivide_factor", 1.0)
        self.sparse_gradients_enabled = p.get("sparse_gradients", False)

        self.zero_config = get_zero_config(p)
        self.mics_shard_size = self.zero_config.mics_shard_size
        self.mics_hierarchial_params_gather = self.zero_config.mics_hierarchical_params_gather
        self.zero_optimization_stage = int(self.zero_config.stage)
        self.zero_enabled = self.zero_optimization_stage > 0
        self.zero_allow_untested_optimizer = p.get("zero_allow_untested_optimizer", False)
        self.zero_force_ds_cpu_optimizer = p.get("zero_force_ds_cpu_optimizer", True)

        self.activation_checkpointing_config = ActivationCheckpointingConfig(**p.get("activation_checkpointing", {}))
        self.comms_config = CommsLoggerConfig(**p.get("comms_logger", {}))
        self.monitor_config = MonitorConfig(tensorboard=TensorBoardConfig(**p.get("tensorboard", {})),
                                            wandb=WandbConfig(**p.get("wandb", {})),
                                            csv_monitor=CSVConfig(**p.get("csv_monitor", {})))
        self.flops_profiler_config = FlopsProfilerConfig(**p.get("flops_profiler", {}))
        self.aio_config = AIOConfig(**p.get("aio", {}))

        fp16 = FP16Config(**p.get("fp16", {}))
        self.fp16_config = fp16
        bf16_dict = p.get("bf16", p.get("bfloat16", {}))
        self.bf16_config = BF16Config(**bf16_dict)
        self.fp16_enabled = fp16.enabled
        self.fp16_auto_cast = fp16.auto_cast
        self.bfloat16_enabled = self.bf16_config.enabled
        self.bfloat16_immediate_grad_update = self.bf16_config.immediate_grad_update
        assert not (self.fp16_enabled and self.bfloat16_enabled), "bf16 and fp16 modes cannot be simultaneously enabled"
        self.fp16_master_weights_and_gradients = fp16.fp16_master_weights_and_grads
        self.amp_config = AMPConfig(**p.get("amp", {}))
        self.amp_enabled = self.amp_config.enabled
        self.amp_params = {k: v for k, v in p.get("amp", {}).items() if k != "enabled"}
        self.loss_scale = fp16.loss_scale
        self.initial_dynamic_scale = 2**fp16.initial_scale_power
        self.dynamic_loss_scale_args = None
        if self.fp16_enabled and fp16.loss_scale == 0:
            self.dynamic_loss_scale_args = {
                "init_scale": 2**fp16.initial_scale_power,
                "scale_window": fp16.loss_scale_window,
                "delayed_shift": fp16.hysteresis,
                "consecutive_hysteresis": fp16.consecutive_hysteresis,
                "min_scale": fp16.min_loss_scale,
            }

        self.gradient_clipping = p.get("gradient_clipping", 0.0)
        opt = p.get("optimizer")
        self.optimizer_name = None
        self.optimizer_params = None
        self.optimizer_legacy_fusion = False
        if opt is not None:
            name = opt.get("type")
            self.optimizer_name = name.lower() if name and name.lower() in DEEPSPEED_OPTIMIZERS else name
            self.optimizer_params = dict(opt.get("params", {}))
            self.optimizer_legacy_fusion = opt.get("legacy_fusion", False)
            if MAX_GRAD_NORM in self.optimizer_params and not self.gradient_clipping:
                self.gradient_clipping = self.optimizer_params.pop(MAX_GRAD_NORM)
        sched = p.get("scheduler")
        self.scheduler_name = sched.get("type") if sched else None
        self.scheduler_params = sched.get("params", {}) if sched else None

        self.wall_clock_breakdown = p.get("wall_clock_breakdown", False) | self.flops_profiler_config.enabled
        self.memory_breakdown = p.get("memory_breakdown", False)
        self.sparse_attention = p.get("sparse_attention")
        self.pipeline = PipelineConfig(**p.get("pipeline", {})).model_dump()
        self.pld_enabled = p.get("progressive_layer_drop", {}).get("enabled", False)
        self.pld_params = {k: v for k, v in p.get("progressive_layer_drop", {}).items() if k != "enabled"}
        self.curriculum_enabled_legacy = p.get("curriculum_learning", {}).get("enabled", False)
        self.curriculum_params_legacy = p.get("curriculum_learning", {})
        self.data_efficiency_config = p.get("data_efficiency", {})
        self.data_efficiency_enabled = self.data_efficiency_config.get("enabled", False)
        ev = p.get("eigenvalue", {})
        self.eigenvalue_enabled = ev.get("enabled", False)
        self.eigenvalue_verbose = ev.get("verbose", False)
        self.eigenvalue_max_iter = ev.get("max_iter", 100)
        self.eigenvalue_tol = ev.get("tol", 1e-2)
        self.eigenvalue_stability = ev.get("stability", 1e-6)
        self.eigenvalue_gas_boundary_resolution = ev.get("gas_boundary_resolution", 1)
        self.eigenvalue_layer_name = ev.get("layer_name", "bert.encoder.layer")
        self.eigenvalue_layer_num = ev.get("layer_num", 0)
        ck = CheckpointConfig(**p.get("checkpoint", {}))
        self.checkpoint_config = ck
        self.checkpoint_tag_validation_enabled = ck.tag_validation.lower() != "ignore"
        self.checkpoint_tag_validation_fail = ck.tag_validation.lower() == "fail"
        self.load_universal_checkpoint = ck.load_universal
        self.use_node_local_storage = ck.use_node_local_storage
        self.checkpoint_parallel_write_pipeline = bool(ck.parallel_write.get("pipeline_stage", False))
        dt = DataTypesConfig(**p.get("data_types", {}))
        self.grad_accum_dtype = dt.grad_accum_dtype
        self.hybrid_engine = HybridEngineConfig(**p.get("hybrid_engine", {}))
        self.elasticity_config = p.get("elasticity", {})
        self.elasticity_enabled = self.elasticity_config.get("enabled", False)
        self.autotuning_config = p.get("autotuning", {})
        self.compression_config = p.get("compression_training", {})
        self.dataloader_drop_last = p.get("dataloader_drop_last", False)
        self.sequence_parallel_config = SequenceParallelConfig(**p.get("sequence_parallel", {}))
        self.sequence_parallel_size = self.sequence_parallel_config.size
        self.use_data_before_expert_parallel_ = p.get("use_data_before_expert_parallel_", False)
        self.graph_harvesting = p.get("graph_harvesting", False)
        self.nebula_config = p.get("nebula", {})

    # --------------------------------------------------------------------------------------- batch solve
    def _configure_train_batch_size(self):
        tb, mb, ga = self.train_batch_size, self.train_micro_batch_size_per_gpu, self.gradient_accumulation_steps
        ws = self.world_size
        if tb is not None and mb is not None and ga is not None:
            pass
        elif tb is not None and mb is not None:
            self.gradient_accumulation_steps = tb // mb // ws
        elif tb is not None and ga is not None:
            self.train_micro_batch_size_per_gpu = tb // ws // ga
        elif mb is not None and ga is not None:
            self.train_batch_size = mb * ga * ws
        elif tb is not None:
            self.gradient_accumulation_steps = 1
            self.train_micro_batch_size_per_gpu = tb // ws
        elif mb is not None:
            self.train_batch_size = mb * ws
            self.gradient_accumulation_steps = 1
        else:
            raise DeepSpeedConfigError(
                "Either train_batch_size or train_micro_batch_size_per_gpu needs to be provided")
        tb, mb, ga = self.train_batch_size, self.train_micro_batch_size_per_gpu, self.gradient_accumulation_steps
        if tb <= 0 or mb <= 0 or ga <= 0:
            raise DeepSpeedConfigError(f"batch parameters must be positive: train_batch_size={tb} "
                                       f"micro_batch={mb} gas={ga}")
        if tb != mb * ga * ws:
            raise DeepSpeedConfigError(
                f"Check batch related parameters. train_batch_size is not equal to micro_batch_per_gpu * "
                f"gradient_acc_step * world_size {tb} != {mb} * {ga} * {ws}")

    def _do_sanity_check(self):
        if self.zero_enabled and self.zero_optimization_stage > int(ZeroStageEnum.max_stage):
            raise DeepSpeedConfigError(f"ZeRO stage must be <= {int(ZeroStageEnum.max_stage)}")
        if self.fp16_master_weights_and_gradients:
            assert self.zero_enabled and self.zero_optimization_stage == 2, \
                "fp16_master_and_gradients requires optimizer to support keeping fp16 master and gradients " \
                "while keeping the optimizer states in fp32. Currently only supported using ZeRO-Offload " \
                "with stage 2"

    # --------------------------------------------------------------------------------------- misc
    @property
    def param_dict(self):
        return self._param_dict

    def print_user_config(self):
        logger.info("  json = {}".format(
            json.dumps(self._param_dict, sort_keys=True, indent=4, cls=ScientificNotationEncoder,
                       separators=(",", ":"))))

    def print(self, name):
        logger.info(f"{name}:")
        for arg in sorted(vars(self)):
            if arg != "_param_dict":
                dots = "." * (29 - len(arg))
                logger.info(f"  {arg} {dots} {getattr(self, arg)}")
        self.print_user_config()
