"""DeepSpeedEngine: the training engine behind `initialize()` (reference `runtime/engine.py:179-3600`).

Same user contract: `loss = engine(batch)`, `engine.backward(loss)`, `engine.step()`, `save_checkpoint`/
`load_checkpoint` with the reference's file names and top-level keys, `train_batch_size()` & friends.

All precision / ZeRO modes run through `FlatZeroOptimizer` (see `runtime/zero/flat_optimizer.py`): stage 0 (bf16 /
fp16 / fp32 data parallel), 1, 2 and 3, with fused gfx950 Adam and RCCL collectives on side streams.
"""
import os
import re
import time
from collections import OrderedDict

import torch
import torch.nn as nn

from .. import comm as dist
from ..accelerator import get_accelerator
from ..checkpoint import constants as CK
from ..parallel import groups
from ..utils.logging import log_dist, logger
from ..utils.timer import (BACKWARD_GLOBAL_TIMER, BACKWARD_MICRO_TIMER, FORWARD_GLOBAL_TIMER, FORWARD_MICRO_TIMER,
                           STEP_GLOBAL_TIMER, STEP_MICRO_TIMER, NoopTimer, SynchronizedWallClockTimer, ThroughputTimer)
from . import lr_schedules
from .checkpoint_engine import AsyncCheckpointEngine, TorchCheckpointEngine
from .config import (ADAGRAD_OPTIMIZER, ADAM_OPTIMIZER, ADAMW_OPTIMIZER, LAMB_OPTIMIZER, LION_OPTIMIZER,
                     ONEBIT_ADAM_OPTIMIZER, ONEBIT_LAMB_OPTIMIZER, SGD_OPTIMIZER, ZERO_ONE_ADAM_OPTIMIZER,
                     DeepSpeedConfig)
from .dataloader import DeepSpeedDataLoader, RepeatingLoader
from .zero.flat_optimizer import FlatZeroOptimizer


def _version():
    from .. import __version__
    return __version__


def split_half_float_double_sparse(tensors):
    """Bucket gradients by dtype for the plain data-parallel reduction: [(dtype name, [tensors])], sparse
    gradients in a bucket of their own (reference `engine.py:121-141`)."""
    from .sparse_tensor import SparseTensor
    buckets = {}
    for t in tensors:
        key = SparseTensor.type() if isinstance(t, SparseTensor) else t.type()
        buckets.setdefault(key, []).append(t)
    return list(buckets.items())


class EngineTimers:
    """Which wall-clock timers the engine reports (reference `engine.py:144-176`): micro-step and global timers of
    forward / backward / reduce / step, all empty when timing is off."""

    def __init__(self, enable_micro_timers, enable_global_timers):
        from ..utils import timer as T
        self.forward_timers, self.backward_timers = [], []
        self.backward_inner_timers, self.backward_reduce_timers = [], []
        self.step_timers, self.global_timers, self.micro_timers = [], [], []
        if enable_micro_timers:
            self.forward_timers += [T.FORWARD_MICRO_TIMER]
            self.backward_timers += [T.BACKWARD_MICRO_TIMER]
            self.backward_inner_timers += [T.BACKWARD_INNER_MICRO_TIMER]
            self.backward_reduce_timers += [T.BACKWARD_REDUCE_MICRO_TIMER]
            self.step_timers += [T.STEP_MICRO_TIMER]
            self.micro_timers += [T.FORWARD_MICRO_TIMER, T.BACKWARD_MICRO_TIMER, T.BACKWARD_INNER_MICRO_TIMER,
                                  T.BACKWARD_REDUCE_MICRO_TIMER, T.STEP_MICRO_TIMER]
        if enable_global_timers:
            self.forward_timers += [T.FORWARD_GLOBAL_TIMER]
            self.backward_timers += [T.BACKWARD_GLOBAL_TIMER]
            self.backward_inner_timers += [T.BACKWARD_INNER_GLOBAL_TIMER]
            self.backward_reduce_timers += [T.BACKWARD_REDUCE_GLOBAL_TIMER]
            self.step_timers += [T.STEP_GLOBAL_TIMER]
            self.global_timers += [T.FORWARD_GLOBAL_TIMER, T.BACKWARD_GLOBAL_TIMER, T.BACKWARD_INNER_GLOBAL_TIMER,
                                   T.BACKWARD_REDUCE_GLOBAL_TIMER, T.STEP_GLOBAL_TIMER]


class DeepSpeedEngine(nn.Module):

    def __init__(self, args, model, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
                 mpu=None, dist_init_required=None, collate_fn=None, config=None, config_class=None,
                 dont_change_device=False):
        super().__init__()
        self.dont_change_device = dont_change_device
        self.client_optimizer = optimizer
        self.client_lr_scheduler = lr_scheduler
        self.training_data = training_data
        self.collate_fn = collate_fn
        self.mpu = mpu
        self.global_steps = 0
        self.global_samples = 0
        self.micro_steps = 0
        self.skipped_steps = 0
        self.gradient_average = True
        self.warn_unscaled_loss = True
        self.losses = None
        self.enable_backward_allreduce = True
        self.checkpoint_engine = None
        self._is_gradient_accumulation_boundary = None
        self.training_dataloader = None
        self.sparse_tensor_module_names = set()
        self.acc = get_accelerator()

        if dist_init_required is not False:
            dist.init_distributed(dist_backend=self.acc.communication_backend_name(),
                                  dist_init_required=dist_init_required)
        self._config = config_class if config_class is not None else DeepSpeedConfig(config, mpu)
        dist.configure(deepspeed_config=self._config)
        self._set_distributed_vars(args)
        self._configure_groups()

        self.monitor = None
        try:
            from ..monitor.monitor import MonitorMaster
            self.monitor = MonitorMaster(self._config.monitor_config)
        except Exception:  # monitor backends are optional
            self.monitor = None

        self.module = model
        self._configure_distributed_model(model)
        self.timers = SynchronizedWallClockTimer() if self.wall_clock_breakdown() else NoopTimer()
        self.tput_timer = ThroughputTimer(batch_size=self.train_batch_size(), steps_per_output=self.steps_per_print())
        if training_data is not None:
            self.training_dataloader = self.deepspeed_io(training_data)

        self.optimizer = None
        self.basic_optimizer = None
        self.lr_scheduler = None
        if model_parameters is None:
            model_parameters = self.module.parameters()
        if optimizer is not None or self._config.optimizer_name is not None:
            self._configure_optimizer(optimizer, model_parameters)
            self._configure_lr_scheduler(lr_scheduler)
        elif self.zero_optimization_stage() == 3:
            # ZeRO-3 inference-style partitioning without an optimizer (reference: DeepSpeedZeRoOffload)
            self._configure_optimizer(torch.optim.SGD(self.module.parameters(), lr=0.0), model_parameters)
        self.flops_profiler = None
        if self._config.flops_profiler_config.enabled:
            from ..profiling.flops_profiler import FlopsProfiler
            self.flops_profiler = FlopsProfiler(self.module, ds_engine=self)
        self._configure_checkpointing()
        self._configure_data_efficiency()
        self._configure_autotuning()
        if self.global_rank == 0 and (self._config.dump_state or self._config.param_dict.get("print_config", False)):
            self._config.print("DeepSpeedEngine configuration")

    # ============================================================================================ data efficiency
    def _configure_data_efficiency(self):
        self.curriculum_scheduler_legacy = None
        self.random_ltd_scheduler = None
        self.compression_scheduler = None
        if self._config.curriculum_enabled_legacy:
            from .data_pipeline.curriculum_scheduler import CurriculumScheduler
            self.curriculum_scheduler_legacy = CurriculumScheduler(self._config.curriculum_params_legacy)
        de = self._config.data_efficiency_config or {}
        rl = de.get("data_routing", {}).get("random_ltd", {})
        if de.get("enabled", False) and rl.get("enabled", False):
            from .data_pipeline.data_routing import RandomLayerTokenDrop, RandomLTDScheduler
            self.random_ltd_scheduler = RandomLTDScheduler(rl)
            for i, m in enumerate(x for x in self.module.modules() if isinstance(x, RandomLayerTokenDrop)):
                m.init_config(rl, self.random_ltd_scheduler, i)
        if self._config.compression_config:
            from ..compression.compress import compression_scheduler
            self.compression_scheduler = compression_scheduler(self.module, self._config.compression_config)
        self._configure_moq()
        self.progressive_layer_drop = None
        if self._config.pld_enabled:
            from .progressive_layer_drop import ProgressiveLayerDrop
            self.progressive_layer_drop = ProgressiveLayerDrop(theta=self._config.pld_params.get("theta", 1.0),
                                                               gamma=self._config.pld_params.get("gamma", 0.001))

    def _configure_moq(self):
        """MoQ (reference `engine.py:1384-1401,1643-1655`): weight quantization with `quantize_weight_in_forward`
        off quantises the 16-bit weights after every optimizer step on a per-weight bit schedule, optionally
        stretched per block by Hessian eigenvalues."""
        self.quantizer, self.eigenvalue, self.block_eigenvalue = None, None, None
        self.gas_boundary_ctr = 0
        c = self._config
        if c.eigenvalue_enabled:
            from .eigenvalue import Eigenvalue
            self.eigenvalue = Eigenvalue(verbose=c.eigenvalue_verbose, max_iter=c.eigenvalue_max_iter,
                                         tol=c.eigenvalue_tol, stability=c.eigenvalue_stability,
                                         gas_boundary_resolution=c.eigenvalue_gas_boundary_resolution,
                                         layer_name=c.eigenvalue_layer_name, layer_num=c.eigenvalue_layer_num)
        wq = (c.compression_config or {}).get("weight_quantization", {}).get("shared_parameters", {})
        if not wq.get("enabled", False) or wq.get("quantize_weight_in_forward", False):
            return
        from .quantize import Quantizer
        self.quantizer = Quantizer(q_groups=wq.get("quantize_groups", 1),
                                   q_mixed_fp16=wq.get("fp16_mixed_quantize", {}).get("enabled", False),
                                   q_change_ratio=wq.get("fp16_mixed_quantize", {}).get("quantize_change_ratio",
                                                                                        0.001),
                                   q_type=wq.get("quantization_type", "symmetric"),
                                   q_rounding=wq.get("rounding", "nearest"), q_verbose=wq.get("quantize_verbose",
                                                                                              False),
                                   q_eigenvalue=c.eigenvalue_enabled,
                                   use_quantizer_kernel=wq.get("quantizer_kernel", False),
                                   layer_num=c.eigenvalue_layer_num if c.eigenvalue_enabled else 0)
        if self.compression_scheduler is not None:
            self.compression_scheduler.moq_external = True
        if self._zero3_partitioned():
            # the step-time quantizer walks module.parameters(), which are empty placeholders once ZeRO-3 has
            # partitioned them: it would silently quantize nothing
            raise NotImplementedError("MoQ weight quantization after the optimizer step (quantize_weight_in_forward: "
                                      "false) is not supported with partitioned ZeRO-3 parameters; use ZeRO stage "
                                      "<= 2 or quantize_weight_in_forward: true")

    def _moq_quantize(self, block_eigenvalue=None):
        if self.quantizer is None or self.compression_scheduler is None or \
                not self.compression_scheduler.weight_quantization_enabled:
            return
        overflow = bool(self.optimizer.overflow) if (self.optimizer is not None and self.fp16_enabled()) else False
        self.quantizer.quantize([list(self.module.parameters())], overflow, self.eigenvalue is not None,
                                block_eigenvalue)

    def _eigenvalue_due(self):
        return (self.eigenvalue is not None and self.quantizer is not None and
                (self.gas_boundary_ctr + 1) % self.eigenvalue.gas_boundary_resolution == 0 and
                self.quantizer.any_precision_switch())

    def _configure_autotuning(self):
        """Autotuning experiment mode (reference engine.py autotuning hooks): report model info, or measure the
        metric between start_profile_step and end_profile_step, write it to metric_path, and end the process."""
        at = (self._config.autotuning_config or {})
        self._autotuning = at if at.get("enabled", False) and (at.get("metric_path") or
                                                              at.get("model_info", {}).get("profile")) else None
        self._at_t0 = None
        if self._autotuning is not None and at.get("model_info", {}).get("profile"):
            import json
            n = sum(p.numel() for p in self.module.parameters())
            path = at.get("model_info_path")
            if self.global_rank == 0 and path:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "w") as f:
                    json.dump({"num_params": n}, f)
            if at.get("metric_path") and self.global_rank == 0:
                os.makedirs(os.path.dirname(at["metric_path"]), exist_ok=True)
                with open(at["metric_path"], "w") as f:
                    json.dump({"num_params": n}, f)
            dist.barrier()
            raise SystemExit(0)

    def _autotuning_step(self):
        import json
        import time
        at = self._autotuning
        start, end = at.get("start_profile_step", 3), at.get("end_profile_step", 5)
        if self.global_steps == start:
            self.acc.synchronize()
            self._at_t0 = time.time()
        elif self.global_steps == end and self._at_t0 is not None:
            self.acc.synchronize()
            dt = (time.time() - self._at_t0) / max(end - start, 1)
            res = {"throughput": self.train_batch_size() / dt, "latency": dt,
                   "flops": None, "micro_batch": self.train_micro_batch_size_per_gpu(),
                   "zero_stage": self.zero_optimization_stage()}
            if self.global_rank == 0:
                os.makedirs(os.path.dirname(at["metric_path"]) or ".", exist_ok=True)
                with open(at["metric_path"], "w") as f:
                    json.dump(res, f)
            dist.barrier()
            raise SystemExit(0)

    def _module_accepts(self, kw):
        import inspect
        try:
            return kw in inspect.signature(self.module.forward).parameters
        except (TypeError, ValueError):
            return False

    def get_data_parallel_rank(self):
        return dist.get_rank(self.seq_data_parallel_group) if self.seq_data_parallel_group is not None else 0

    # ============================================================================================ setup
    def _set_distributed_vars(self, args):
        self.local_rank = int(os.environ.get("LOCAL_RANK", getattr(args, "local_rank", 0) or 0))
        if self.acc.device_name() != "cpu" and self.acc.is_available():
            self.acc.set_device(self.local_rank % max(self.acc.device_count(), 1))
            self.device = torch.device("cuda", self.acc.current_device())
        else:
            self.device = torch.device("cpu")
        self.world_size = dist.get_world_size()
        self.global_rank = dist.get_rank()
        from ..utils.fault_injection import FaultInjector
        fi = FaultInjector(self.global_rank)
        self._fault_injector = fi if fi.active else None

    def _configure_groups(self):
        sp = self._config.sequence_parallel_size
        if self.mpu is not None:
            groups.mpu = self.mpu
        elif sp > 1 and groups._get_sequence_parallel_group() is None:
            groups.initialize_sequence_parallel(sp)
        self.sequence_parallel_size = groups._get_sequence_parallel_world_size()
        self.seq_data_parallel_group = groups._get_sequence_data_parallel_group()
        self.seq_dp_world_size = dist.get_world_size(self.seq_data_parallel_group)
        self.dp_world_size = groups._get_data_parallel_world_size()
        self.mp_world_size = groups._get_model_parallel_world_size()

    def _dtype(self):
        if self.fp16_enabled():
            return torch.float16
        if self.bfloat16_enabled():
            return torch.bfloat16
        return torch.float32

    def _configure_distributed_model(self, model):
        already_partitioned = any(hasattr(p, "ds_tensor") for p in model.parameters())
        dtype = self._dtype()
        if not already_partitioned:
            if not self.dont_change_device:
                model.to(self.device)
            if dtype != torch.float32:
                for p in model.parameters():
                    if p.is_floating_point():
                        p.data = p.data.to(dtype)
                for b in model.buffers():
                    pass  # buffers (e.g. fp32 rope tables) keep their dtype
            self._broadcast_model()

    @torch.no_grad()
    def _broadcast_model(self):
        if dist.get_world_size() == 1:
            return
        from ..moe.utils import is_moe_param
        src = groups._get_broadcast_src_rank()
        for p in self.module.parameters():
            if not (torch.is_tensor(p) and p.numel() > 0):
                continue
            if is_moe_param(p):
                # experts differ across EP ranks: replicate only within the expert-data-parallel group
                dist.broadcast(p.data, groups._get_expert_broadcast_src_rank(p.group_name),
                               group=groups._get_expert_data_parallel_group(p.group_name))
            else:
                dist.broadcast(p.data, src, group=self.seq_data_parallel_group)

    # ============================================================================================ optimizer
    def _configure_basic_optimizer(self, model_parameters):
        name = self._config.optimizer_name
        params = dict(self._config.optimizer_params or {})
        params.pop("torch_adam", None)
        adam_w_mode = params.pop("adam_w_mode", True)
        if name in (ADAM_OPTIMIZER, ADAMW_OPTIMIZER):
            from ..ops.adam import FusedAdam
            if name == ADAMW_OPTIMIZER:
                adam_w_mode = True
            elif "adam_w_mode" not in (self._config.optimizer_params or {}):
                adam_w_mode = True if name == ADAMW_OPTIMIZER else adam_w_mode
            return FusedAdam(model_parameters, adam_w_mode=adam_w_mode, **params)
        if name == LAMB_OPTIMIZER:
            from ..ops.lamb import FusedLamb
            return FusedLamb(model_parameters, **params)
        if name == LION_OPTIMIZER:
            from ..ops.lion import FusedLion
            return FusedLion(model_parameters, **params)
        if name == ADAGRAD_OPTIMIZER:
            return torch.optim.Adagrad(model_parameters, **params)
        if name == SGD_OPTIMIZER:
            return torch.optim.SGD(model_parameters, **params)
        if name in (ONEBIT_ADAM_OPTIMIZER, ZERO_ONE_ADAM_OPTIMIZER, ONEBIT_LAMB_OPTIMIZER):
            from ..runtime.fp16.onebit import build_onebit_optimizer
            return build_onebit_optimizer(name, model_parameters, self, params)
        # any torch.optim class by name
        cls = getattr(torch.optim, name, None)
        if cls is None:
            raise ValueError(f"Unknown optimizer {name}")
        return cls(model_parameters, **params)

    def _configure_optimizer(self, client_optimizer, model_parameters):
        from ..moe.utils import has_moe_layers, split_params_into_different_moe_groups_for_optimizer
        self.has_moe_layers, self.num_experts = has_moe_layers(self.module)
        if self.has_moe_layers:
            if client_optimizer is None or not isinstance(client_optimizer, torch.optim.Optimizer):
                mp = list(model_parameters)
                if mp and torch.is_tensor(mp[0]):
                    mp = [{"params": mp}]
                model_parameters = split_params_into_different_moe_groups_for_optimizer(mp)
            elif not any(g.get("moe", False) for g in client_optimizer.param_groups):
                new = split_params_into_different_moe_groups_for_optimizer(client_optimizer.param_groups)
                client_optimizer.param_groups = []
                for g in new:
                    client_optimizer.add_param_group(g)
        if client_optimizer is None:
            basic = self._configure_basic_optimizer(model_parameters)
        elif isinstance(client_optimizer, torch.optim.Optimizer):
            basic = client_optimizer
        else:
            basic = client_optimizer(model_parameters)
        self.basic_optimizer = basic
        stage = self.zero_optimization_stage()
        dtype = self._dtype()
        zc = self._config.zero_config
        self._check_optimizer_options(basic, stage, zc)
        if getattr(zc, "memory_efficient_linear", True) and next(self.module.parameters()).is_cuda:
            # every nn.Linear on the training linear of ops/linear.py (K-major weight-gradient GEMMs; the ZeRO-3
            # coordinator installs the same function for partitioned runs)
            from .zero.linear import install_zero3_linear
            install_zero3_linear(self.module)
        # sparse embedding gradients (reference `runtime/engine.py:325-327,2447-2518`): with `sparse_gradients` the
        # weight gradient of every nn.Embedding / nn.EmbeddingBag travels as (row indices, rows) in an all-gather
        # instead of a dense [vocab, hidden] reduction
        sparse_params = set()
        if self._config.sparse_gradients_enabled:
            for name, m in self.module.named_modules():
                if isinstance(m, (nn.Embedding, nn.EmbeddingBag)):
                    self.sparse_tensor_module_names.add(name + ".weight")
                    sparse_params.add(id(m.weight))
                    log_dist(f"Will reduce the gradient of {name}.weight as a sparse tensor", ranks=[0])
        comm_dtype = self._config.communication_data_type
        if self.sequence_parallel_size > 1:
            # reference `runtime/engine.py:1144-1145`: under Ulysses the gradient reduction over the sequence x data
            # group runs in seq_parallel_communication_data_type (fp32 unless configured)
            comm_dtype = self._config.seq_parallel_communication_data_type
        self.optimizer = FlatZeroOptimizer(basic, self.module, self._config, dp_group=self.seq_data_parallel_group,
                                           stage=stage, mpu=self.mpu, clip_grad=self.gradient_clipping(),
                                           dtype=dtype, communication_data_type=comm_dtype,
                                           zero_config=self._config.zero_config, timers=None,
                                           gradient_accumulation_steps=self.gradient_accumulation_steps(),
                                           sparse_params=sparse_params)

    def _check_optimizer_options(self, basic, stage, zc):
        """Config keys that gate optimizer choices (reference `runtime/engine.py:1219-1265,1475-1500`): an optimizer
        ZeRO was not validated with needs `zero_allow_untested_optimizer`. Optimizer offload steps the host partitions
        with the native CPU Adam, so a client `torch.optim.Adam` / `AdamW` / `DeepSpeedCPUAdam` is taken over by the
        flat Adam path (same update rule, hyper-parameters read from its param groups) and any other optimizer is
        refused up front, whatever `zero_force_ds_cpu_optimizer` says: there is no torch fallback for host shards."""
        from ..ops.adagrad.cpu_adagrad import DeepSpeedCPUAdagrad
        from ..ops.adam.cpu_adam import DeepSpeedCPUAdam
        from ..ops.adam.fused_adam import FusedAdam
        from ..ops.lamb.fused_lamb import FusedLamb
        from ..ops.lion.cpu_lion import DeepSpeedCPULion
        from ..ops.lion.fused_lion import FusedLion
        from .zero.utils import ZeRORuntimeException
        cfg = self._config
        flat_adam = isinstance(basic, FusedAdam) or getattr(basic, "_ds_flat_adam", False)
        tested = (torch.optim.Adam, torch.optim.AdamW, FusedAdam, DeepSpeedCPUAdam, DeepSpeedCPUAdagrad,
                  DeepSpeedCPULion, FusedLion, FusedLamb, torch.optim.Adagrad)
        if stage > 0 and not isinstance(basic, tested) and not flat_adam and not cfg.zero_allow_untested_optimizer:
            raise ZeRORuntimeException(
                f"You are using an untested ZeRO Optimizer ({type(basic).__name__}). Please add "
                f"<\"zero_allow_untested_optimizer\": true> in the configuration file to use it.")
        off = getattr(zc, "offload_optimizer", None)
        offloading = off is not None and str(getattr(off.device, "value", off.device)) in ("cpu", "nvme")
        if offloading and not flat_adam:
            plain = all(not g.get(k, False) for g in basic.param_groups for k in ("amsgrad", "maximize"))
            if isinstance(basic, DeepSpeedCPUAdam):
                basic._ds_flat_adam = True  # already carries adam_w_mode
            elif isinstance(basic, torch.optim.AdamW) and plain:
                basic._ds_flat_adam, basic.adam_w_mode = True, True
            elif isinstance(basic, torch.optim.Adam) and plain:
                basic._ds_flat_adam, basic.adam_w_mode = True, False
            else:
                hint = "" if cfg.zero_force_ds_cpu_optimizer else \
                    " (zero_force_ds_cpu_optimizer=false does not help: host shards have no torch-stepped fallback)"
                raise ZeRORuntimeException(
                    f"optimizer offload steps the host partitions with the native CPU Adam; "
                    f"{type(basic).__name__} cannot be offloaded. Use Adam / AdamW / DeepSpeedCPUAdam{hint}.")
        if cfg.fp16_master_weights_and_gradients:
            raise NotImplementedError("fp16.fp16_master_weights_and_grads: master weights are kept in fp32 (or as a "
                                      "bf16 weight + 16-bit residual with bf16.split_master_weights)")
        if cfg.mics_hierarchial_params_gather:
            log_dist("mics_hierarchical_params_gather: used for MiCS shard groups that span several nodes (two-level "
                     "all-gather); a shard group inside one xGMI node gathers in one step", ranks=[0])
        for key, default in (("round_robin_gradients", False), ("legacy_stage1", False),
                             ("pipeline_loading_checkpoint", False), ("use_multi_rank_bucket_allreduce", True),
                             ("allgather_partitions", True), ("contiguous_gradients", True)):
            if getattr(zc, key, default) != default:
                log_dist(f"zero_optimization.{key}={getattr(zc, key)}: no effect here (gradients always live in "
                         "contiguous flat buffers reduced per group; partitions are gathered per group)", ranks=[0])
        if cfg.graph_harvesting:
            log_dist("graph_harvesting: the gradient-norm and clipping passes are already single multi-tensor "
                     "launches (sumsq_multi, clip folded into the Adam kernel's gradient scale); nothing to capture",
                     ranks=[0])
        if cfg.bfloat16_immediate_grad_update:
            log_dist("bf16.immediate_grad_update: gradients are always folded into the flat reduction buffers from "
                     "the backward hooks (the immediate form)", ranks=[0])

    def _configure_lr_scheduler(self, client_lr_scheduler):
        name = self._config.scheduler_name
        if name is not None:
            cls = lr_schedules.SCHEDULERS.get(name) or getattr(torch.optim.lr_scheduler, name)
            self.lr_scheduler = cls(self.optimizer.optimizer, **(self._config.scheduler_params or {}))
        elif client_lr_scheduler is not None:
            self.lr_scheduler = client_lr_scheduler(self.optimizer.optimizer) if callable(client_lr_scheduler) and \
                not hasattr(client_lr_scheduler, "step") else client_lr_scheduler
        else:
            self.lr_scheduler = None

    def _configure_checkpointing(self):
        self.checkpoint_engine = AsyncCheckpointEngine() if self._config.nebula_config.get("enabled", False) \
            else TorchCheckpointEngine()
        # `checkpoint.use_node_local_storage` (reference `runtime/engine.py:933-941,3070`): every node has its own
        # disk, so local rank 0 of EVERY node writes the model file, creates the folder and the `latest` marker
        self._ckpt_lead_rank = self.local_rank if self._config.use_node_local_storage else dist.get_rank()
        lead = self.local_rank if self._config.use_node_local_storage else dist.get_rank(self.seq_data_parallel_group)
        self.save_non_zero_checkpoint = lead == 0 or self.zero_optimization_stage() == 3
        self.save_zero_checkpoint = self.optimizer is not None

    # ============================================================================================ config accessors
    @property
    def config(self):
        return self._config.param_dict

    def train_batch_size(self):
        return self._config.train_batch_size

    def train_micro_batch_size_per_gpu(self):
        return self._config.train_micro_batch_size_per_gpu

    def gradient_accumulation_steps(self):
        return self._config.gradient_accumulation_steps

    def set_train_batch_size(self, train_batch_size):
        if train_batch_size % (self.train_micro_batch_size_per_gpu() * self.dp_world_size) != 0:
            raise ValueError("Train batch size must be divisible by micro-batch data parallelism")
        new_gas = train_batch_size // (self.train_micro_batch_size_per_gpu() * self.dp_world_size)
        self._config.train_batch_size = train_batch_size
        self._config.gradient_accumulation_steps = new_gas
        if self.optimizer is not None:
            self.optimizer.gas = new_gas

    def steps_per_print(self):
        return self._config.steps_per_print

    def zero_optimization(self):
        return self._config.zero_enabled

    def zero_optimization_stage(self):
        return self._config.zero_optimization_stage

    def zero_optimization_partition_gradients(self):
        return self.zero_optimization_stage() >= 2

    def zero_optimization_partition_weights(self):
        return self.zero_optimization_stage() >= 3

    def zero_offload_optimizer(self):
        return self._config.zero_config.offload_optimizer

    def zero_offload_param(self):
        return self._config.zero_config.offload_param

    def fp16_enabled(self):
        return self._config.fp16_enabled

    def bfloat16_enabled(self):
        return self._config.bfloat16_enabled

    def amp_enabled(self):
        return self._config.amp_enabled

    def gradient_clipping(self):
        return self._config.gradient_clipping

    def wall_clock_breakdown(self):
        return self._config.wall_clock_breakdown

    def memory_breakdown(self):
        return self._config.memory_breakdown

    def get_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups] if self.optimizer else []

    def get_mom(self):
        return [g.get("betas", (g.get("momentum", 0), ))[0] for g in self.optimizer.param_groups]

    def get_global_grad_norm(self):
        return self.optimizer.get_global_grad_norm() if self.optimizer else None

    @property
    def loss_scale(self):
        return self.optimizer.loss_scale if self.optimizer else 1.0

    def get_data_parallel_group(self):
        return self.seq_data_parallel_group

    def is_gradient_accumulation_boundary(self):
        if self._is_gradient_accumulation_boundary is None:
            return (self.micro_steps + 1) % self.gradient_accumulation_steps() == 0
        return self._is_gradient_accumulation_boundary

    def set_gradient_accumulation_boundary(self, is_boundary):
        self._is_gradient_accumulation_boundary = is_boundary

    # ============================================================================================ data
    def curriculum_learning_enabled(self):
        de = self._config.data_efficiency_config or {}
        cl = de.get("data_sampling", {}).get("curriculum_learning", {})
        return bool(de.get("enabled", False) and de.get("data_sampling", {}).get("enabled", False) and
                    cl.get("enabled", False))

    def deepspeed_io(self, dataset, batch_size=None, route="train", pin_memory=True, data_sampler=None,
                     collate_fn=None, num_local_io_workers=None):
        """Reference `runtime/engine.py:1686-1745`: the engine's loader over the data-parallel ranks; eval / predict
        routes read in order; with `data_efficiency.data_sampling.curriculum_learning` on, batches come from the
        curriculum `DeepSpeedDataSampler`."""
        dp_world, dp_rank = self.dp_world_size, groups._get_data_parallel_rank()
        if self.mpu is not None:
            dp_world, dp_rank = self.mpu.get_data_parallel_world_size(), self.mpu.get_data_parallel_rank()
        if data_sampler is None and route in ("predict", "eval"):
            data_sampler = torch.utils.data.DistributedSampler(dataset, num_replicas=dp_world, rank=dp_rank,
                                                               shuffle=False)
        dl_config = {}
        if self.curriculum_learning_enabled() and route == "train":
            de = self._config.data_efficiency_config
            dl_config = {"curriculum_learning": True, "data_efficiency": de,
                         "data_parallel_group": groups._get_data_parallel_group(),
                         "gradient_accumulation_steps": self.gradient_accumulation_steps(),
                         "global_rank": self.global_rank,
                         "data_sampling_num_workers": de.get("data_sampling", {}).get("num_workers", 0)}
        return DeepSpeedDataLoader(dataset, batch_size or self.train_micro_batch_size_per_gpu(),
                                   pin_memory and self.device.type == "cuda", self.local_rank,
                                   self.tput_timer if route == "train" else None,
                                   collate_fn=collate_fn or self.collate_fn,
                                   num_local_io_workers=num_local_io_workers, data_sampler=data_sampler,
                                   data_parallel_world_size=dp_world, data_parallel_rank=dp_rank,
                                   dataloader_drop_last=self._config.dataloader_drop_last,
                                   deepspeed_dataloader_config=dl_config)

    def set_data_post_process_func(self, post_process_func):
        if self.training_dataloader is not None:
            self.training_dataloader.post_process_func = post_process_func

    # ============================================================================================ train loop
    def train(self, mode=True):
        self.module.train(mode)
        return self

    def eval(self):
        self.module.eval()
        return self

    def forward(self, *inputs, **kwargs):
        if self.flops_profiler is not None and self.global_steps == self._config.flops_profiler_config.profile_step \
                and self.is_gradient_accumulation_boundary():
            self.flops_profiler.start_profile(ignore_list=None)
        self.timers(FORWARD_MICRO_TIMER).start()
        if self.training and self.optimizer is not None:
            self.optimizer.is_gradient_accumulation_boundary = self.is_gradient_accumulation_boundary()
        if self.training and self.curriculum_scheduler_legacy is not None:
            # legacy curriculum (reference engine.py forward): sequence-length difficulty handed to the model
            d = self.curriculum_scheduler_legacy.update_difficulty(self.global_steps + 1)
            if self._module_accepts("curriculum_seqlen"):
                kwargs["curriculum_seqlen"] = d
        if self.global_steps == 0 and self.micro_steps == 0 and self.compression_scheduler is not None and \
                self.module.training:
            # techniques with schedule_offset 0 switch on before the first forward (reference engine.py:1796-1807)
            self.compression_scheduler.step(step_zero_check=0)
            self._moq_quantize()
        if self.module.training and self.progressive_layer_drop is not None:
            kwargs.update(self.progressive_layer_drop.get_state())
        if self.optimizer is not None:
            self.optimizer.offload_pre_forward()
        if self._config.fp16_auto_cast:
            # reference `runtime/engine.py:1808-1810`: floating-point inputs follow the fp16 module
            inputs = self._cast_inputs_half(inputs)
            kwargs = self._cast_inputs_half(kwargs)
        loss = self.module(*inputs, **kwargs)
        self.timers(FORWARD_MICRO_TIMER).stop()
        return loss

    @staticmethod
    def _cast_inputs_half(inputs):
        """Floating-point tensors anywhere inside tuples / lists / dicts become fp16 (reference
        `runtime/engine.py:1757-1772`)."""
        cast = DeepSpeedEngine._cast_inputs_half
        if isinstance(inputs, (list, tuple)):
            return type(inputs)(cast(v) for v in inputs)
        if isinstance(inputs, dict):
            return {k: cast(v) for k, v in inputs.items()}
        if torch.is_tensor(inputs) and inputs.is_floating_point():
            return inputs.half()
        return inputs

    def _scale_loss_by_gas(self, loss):
        gas = self.gradient_accumulation_steps()
        if gas > 1:
            if torch.is_tensor(loss):
                return loss / gas
            if isinstance(loss, (list, tuple)):
                return type(loss)(l / gas for l in loss)
        return loss

    def backward(self, loss, allreduce_gradients=True, release_loss=False, retain_graph=False, scale_wrt_gas=True):
        assert self.optimizer is not None, "must provide an optimizer to call backward()"
        self.timers(BACKWARD_MICRO_TIMER).start()
        if scale_wrt_gas:
            loss = self._scale_loss_by_gas(loss)
        if self.monitor is not None and self.monitor.enabled and self.global_rank == 0 and \
                self.is_gradient_accumulation_boundary():
            self.monitor.write_events([("Train/Samples/train_loss", float(loss.detach()) *
                                        self.gradient_accumulation_steps(), self.global_samples)])
        self.optimizer.is_gradient_accumulation_boundary = self.is_gradient_accumulation_boundary()
        if self.is_gradient_accumulation_boundary() and self._eigenvalue_due():
            # Hessian power iteration on this micro-batch's graph before the regular backward consumes it
            log_dist("computing eigenvalue...", ranks=[0])
            self.block_eigenvalue = self.eigenvalue.compute_block_eigenvalue(
                self.module, loss=loss, device=self.device, scale=float(self.optimizer.cur_scale))
            retain_graph = True
        self.optimizer.backward(loss, retain_graph=retain_graph)
        self.timers(BACKWARD_MICRO_TIMER).stop()
        return loss

    def allreduce_gradients(self, bucket_size=None):
        """Kept for API parity: reduction already happened in `backward` (bucketed on the comm stream)."""
        return

    # ---- explicit gradient reductions over module `.grad`s (reference `engine.py:2326-2518`). The engine's own
    # path reduces inside the flat-group optimizer; these serve code that drives the reduction itself (custom
    # loops, engines built without an optimizer).
    def allreduce_bucket(self, bucket, dp_group=None, dp_world_size=None):
        """All-reduce a list of same-dtype dense tensors as ONE flat buffer; returns the averaged flat tensor."""
        from torch._utils import _flatten_dense_tensors
        group = dp_group if dp_group is not None else self.seq_data_parallel_group
        world = dp_world_size or dist.get_world_size(group)
        flat = _flatten_dense_tensors(bucket)
        comm_dtype = getattr(self, "communication_data_type", None)
        comm_dtype = comm_dtype() if callable(comm_dtype) else comm_dtype
        send = flat.to(comm_dtype) if comm_dtype is not None and comm_dtype != flat.dtype else flat
        pre = float(self._config.gradient_predivide_factor or 1.0) if not self._config.prescale_gradients else world
        if pre != 1.0:
            send.mul_(1.0 / pre)
        dist.all_reduce(send, group=group)
        post = world / pre
        if post != 1.0:
            send.mul_(1.0 / post)
        if send is not flat:
            flat.copy_(send)
        return flat

    def allreduce_and_copy(self, small_bucket, dp_group=None, dp_world_size=None):
        from torch._utils import _unflatten_dense_tensors
        flat = self.allreduce_bucket(small_bucket, dp_group, dp_world_size)
        for buf, synced in zip(small_bucket, _unflatten_dense_tensors(flat, small_bucket)):
            buf.copy_(synced)

    def allreduce_no_retain(self, bucket, dp_group=None, numel_per_bucket=500000000, dp_world_size=None):
        small, numel = [], 0
        for t in bucket:
            small.append(t)
            numel += t.numel()
            if numel > numel_per_bucket:
                self.allreduce_and_copy(small, dp_group, dp_world_size)
                small, numel = [], 0
        if small:
            self.allreduce_and_copy(small, dp_group, dp_world_size)

    def sparse_all_gather(self, value, dp_group=None):
        """Concatenation of every rank's rows of a 1-D / 2-D tensor whose leading size differs per rank."""
        group = dp_group if dp_group is not None else self.seq_data_parallel_group
        world = dist.get_world_size(group)
        sizes = self.all_gather_scalar(value.shape[0], group)
        width = max(sizes)
        pad = torch.zeros((width, ) + tuple(value.shape[1:]), dtype=value.dtype, device=value.device)
        pad[:value.shape[0]].copy_(value)
        out = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(out, pad, group=group)
        return [o[:n] for o, n in zip(out, sizes)]

    def all_gather_scalar(self, value, dp_group=None):
        group = dp_group if dp_group is not None else self.seq_data_parallel_group
        world = dist.get_world_size(group)
        dev = self.device if dist.get_backend(group) != "gloo" else "cpu"
        t = torch.tensor([int(value)], dtype=torch.long, device=dev)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return [int(o.item()) for o in out]

    def sparse_allreduce(self, sparse, dp_group=None, dp_world_size=None):
        """Average a `SparseTensor` across ranks: indices and rows of every rank concatenated, rows divided by the
        group size (duplicates add up when the tensor is made dense)."""
        group = dp_group if dp_group is not None else self.seq_data_parallel_group
        world = dp_world_size or dist.get_world_size(group)
        sparse.values = sparse.values / world
        sparse.indices = torch.cat(self.sparse_all_gather(sparse.indices, group))
        sparse.values = torch.cat(self.sparse_all_gather(sparse.values, group))
        return sparse

    def sparse_allreduce_bucket(self, bucket, dp_group=None, dp_world_size=None):
        return [self.sparse_allreduce(s, dp_group, dp_world_size) for s in bucket]

    def sparse_allreduce_no_retain(self, bucket, dp_group=None, dp_world_size=None):
        for s in self.sparse_allreduce_bucket(bucket, dp_group, dp_world_size):
            if s.orig_dense_tensor is not None:
                s.orig_dense_tensor.data = s.to_dense() if not s.orig_dense_tensor.is_sparse else s.to_coo_tensor()

    def buffered_allreduce_fallback(self, grads=None, elements_per_buffer=500000000):
        """All-reduce (average) the module's gradients bucket by bucket, per dtype; embedding gradients listed in
        `sparse_tensor_module_names` travel as (indices, rows)."""
        from .sparse_tensor import SparseTensor
        if grads is None:
            grads = []
            sparse_names = set(getattr(self, "sparse_tensor_module_names", ()) or ())
            for name, p in self.module.named_parameters():
                if p.grad is None:
                    continue
                if name in sparse_names and not p.grad.is_sparse and p.grad.dim() == 2:
                    st = SparseTensor(p.grad.data)
                    st.orig_dense_tensor = p.grad
                    grads.append(st)
                else:
                    grads.append(p.grad.data)
        for kind, bucket in split_half_float_double_sparse(grads):
            if kind == SparseTensor.type():
                self.sparse_allreduce_no_retain(bucket)
            else:
                self.allreduce_no_retain(bucket, numel_per_bucket=elements_per_buffer)

    def clip_fp32_gradients(self):
        from .utils import clip_grad_norm_
        clip_grad_norm_(parameters=self.module.parameters(), max_norm=self.gradient_clipping(), mpu=self.mpu)

    # ---- further accessors
    def is_elastic_model_parallel_supported(self):
        return self.elasticity_enabled() and self._config.elasticity_config.get("version", 0.1) >= 0.2 \
            if hasattr(self._config, "elasticity_config") else False

    def flops_profiler_recompute_fwd_factor(self):
        return getattr(self._config.flops_profiler_config, "recompute_fwd_factor", 0.0)

    def autotuning_model_info_path(self):
        return (self._config._param_dict.get("autotuning", {})).get("model_info_path")

    def autotuning_profile_model_info(self):
        at = self._config._param_dict.get("autotuning", {})
        return bool(at.get("enabled", False) and (at.get("model_info") or {}).get("profile", False))

    def quantize_training(self):
        q = getattr(self, "quantizer", None)
        return q is not None

    def random_ltd_initialize(self):
        return getattr(self, "random_ltd_scheduler", None)

    def is_first_weights_partition_group(self):
        """Does this rank belong to the first replica of the partitioned weights? (MiCS / hpZ replicate them)"""
        opt = self.optimizer
        replicas = getattr(opt, "mics_replica_group", None)
        return True if replicas is None else dist.get_rank(replicas) == 0

    @staticmethod
    def load_moe_state_dict(checkpoint_path, tag, state_dict, old_moe_load, model=None, mpu=None, num_experts=1,
                            checkpoint_engine=None):
        """Merge the per-expert checkpoint files of `tag` into `state_dict` (see `_load_moe_experts`)."""
        import glob
        import os
        for f in sorted(glob.glob(os.path.join(checkpoint_path, str(tag), "layer_*_expert_*_mp_rank_*_model_states.pt"))):
            state_dict.update(torch.load(f, map_location="cpu", weights_only=True))
        return state_dict

    def zero_grad(self):
        self.module.zero_grad(set_to_none=False)

    def step(self, lr_kwargs=None):
        self.timers(STEP_MICRO_TIMER).start()
        self._step_applied = False
        if self.is_gradient_accumulation_boundary():
            self.gas_boundary_ctr += 1
            from .activation_checkpointing import checkpointing as _ckpt
            if _ckpt.CONTIGUOUS_CHECKPOINTING:
                _ckpt.reset()  # every checkpoint of this step has been consumed: refill the buffers from slot 0
            if self.progressive_layer_drop is not None:
                self.progressive_layer_drop.update_state(self.global_steps)
            if self.optimizer is not None:
                self.optimizer.step()
                overflow = self.optimizer.overflow
                self._step_applied = not overflow
                if overflow:
                    self.skipped_steps += 1
                elif self.lr_scheduler is not None:
                    self.lr_scheduler.step(**(lr_kwargs or {}))
                if self.optimizer.coordinator is not None:
                    self.optimizer.coordinator.reset_step()
                use_ev = self.eigenvalue is not None and \
                    self.gas_boundary_ctr % self.eigenvalue.gas_boundary_resolution == 0
                self._moq_quantize(self.block_eigenvalue if use_ev else None)
            self.global_steps += 1
            self.global_samples += self.train_batch_size()
            if self.compression_scheduler is not None:
                self.compression_scheduler.step(self.global_steps)
            if self._autotuning is not None:
                self._autotuning_step()
            if self.random_ltd_scheduler is not None:
                self.random_ltd_scheduler.update_seq(self.global_steps)
            if self.flops_profiler is not None and self.flops_profiler.started:
                self.flops_profiler.stop_profile()
                self.flops_profiler.print_model_profile(profile_step=self.global_steps)
                self.flops_profiler.end_profile()
            if self.monitor is not None and self.monitor.enabled and self.global_rank == 0:
                ev = [("Train/Samples/lr", self.get_lr()[0], self.global_samples)]
                if self.fp16_enabled():
                    ev.append(("Train/Samples/loss_scale", self.optimizer.loss_scale, self.global_samples))
                self.monitor.write_events(ev)
            if self.global_steps % self.steps_per_print() == 0 and self.global_rank == 0:
                log_dist(f"step={self.global_steps}, skipped={self.skipped_steps}, lr={self.get_lr()}", ranks=[0])
            if self.global_steps % self.steps_per_print() == 0 and self.wall_clock_breakdown() and \
                    self.optimizer is not None and self.optimizer.coordinator is not None:
                self.optimizer.coordinator.profiler.log_events()
                self.optimizer.coordinator.profiler.reset_events()
            if self._fault_injector is not None:
                self._fault_injector.on_step(self.global_steps)
        self.micro_steps += 1
        self.timers(STEP_MICRO_TIMER).stop()

    # ============================================================================================ checkpoints
    def _get_ckpt_name(self, checkpoints_path, tag, mp_placeholder=None):
        mp_rank = 0 if self.mpu is None else self.mpu.get_model_parallel_rank()
        mp_str = mp_placeholder if mp_placeholder is not None else f"{mp_rank:02d}"
        if self.zero_optimization_partition_weights():
            dp_rank = dist.get_rank(self.seq_data_parallel_group)
            return os.path.join(checkpoints_path, str(tag), f"{CK.ZERO_FILE_PREFIX}{dp_rank}_mp_rank_{mp_str}"
                                f"{CK.MODEL_FILE_SUFFIX}")
        return os.path.join(checkpoints_path, str(tag), f"{CK.MODEL_FILE_PREFIX}{mp_str}{CK.MODEL_FILE_SUFFIX}")

    def _get_zero_ckpt_name(self, checkpoints_path, tag):
        mp_rank = 0 if self.mpu is None else self.mpu.get_model_parallel_rank()
        dp_rank = dist.get_rank(self.seq_data_parallel_group)
        prefix = CK.BF16_ZERO_FILE_PREFIX if self.bfloat16_enabled() else CK.ZERO_FILE_PREFIX
        return os.path.join(checkpoints_path, str(tag), f"{prefix}{dp_rank}_mp_rank_{mp_rank:02d}{CK.OPTIM_FILE_SUFFIX}")

    def module_state_dict(self, destination=None, prefix="", keep_vars=False, exclude_frozen_parameters=False):
        """The module's state dict as it stands (reference `runtime/engine.py:2520`): under ZeRO-3 the partitioned
        parameters are empty placeholders — their values live in the per-rank optimizer shards, which is what
        `save_checkpoint` writes and `load_checkpoint` restores from. Use `save_16bit_model` (or
        `consolidated_16bit_state_dict`) for a full 16-bit copy."""
        sd = self.module.state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)
        if exclude_frozen_parameters:
            for n, p in self.module.named_parameters():
                if not p.requires_grad and n in sd:
                    del sd[n]
        return sd

    def _zero3_partitioned(self):
        opt = self.optimizer
        return self.zero_optimization_partition_weights() and opt is not None and \
            any((not g.persistent) or g.partition for g in getattr(opt, "all_groups", getattr(opt, "groups", [])))

    @torch.no_grad()
    def consolidated_16bit_state_dict(self, exclude_frozen_parameters=False, rank0_only=True):
        """Full 16-bit state dict gathered ONE flat group at a time (reference `runtime/engine.py:3477-3592`
        `_zero3_consolidated_16bit_state_dict`): every rank joins each group's all-gather, the gathering rank copies
        the group's parameters to host memory, and the device buffer is dropped before the next group — so no rank
        ever holds more than one gathered group on its GPU. Returns the dict on rank 0 (every rank when
        rank0_only=False), None elsewhere."""
        if not self._zero3_partitioned():
            sd = self.module_state_dict(exclude_frozen_parameters=exclude_frozen_parameters)
            return OrderedDict((k, v.detach().cpu().clone()) for k, v in sd.items())
        opt = self.optimizer
        opt.join_offload()
        keep = (not rank0_only) or dist.get_rank() == 0
        names = {id(p): n for n, p in self.module.named_parameters()}
        out = OrderedDict()
        for g in opt.all_groups:
            if g.persistent and g.full is not None:
                full = g.full
            else:
                shard = g.shard if g.shard.device == opt.device else g.shard.to(opt.device, non_blocking=True)
                full = torch.empty(g.padded, dtype=g.shard.dtype, device=opt.device)
                if g.partition:
                    dist.all_gather_into_tensor(full, shard.contiguous(), group=g.dp_group)
                else:
                    full.copy_(shard)
            if keep:
                for i, p in enumerate(g.params):
                    n = names.get(id(p))
                    if n is not None:
                        out[n] = full[g.offsets[i]:g.offsets[i] + g.numels[i]].view(p.ds_shape).cpu().clone()
            del full
        if keep:
            for n, t in self.module.state_dict().items():  # buffers and parameters the optimizer does not own
                if n not in out and not (exclude_frozen_parameters and n in names.values() and
                                         not dict(self.module.named_parameters())[n].requires_grad):
                    out[n] = t.detach().cpu().clone()
            ordered = OrderedDict((k, out[k]) for k in self.module.state_dict().keys() if k in out)
            return ordered
        return None

    def _param_shapes(self):
        """One ordered name -> full shape dict per optimizer param group, parameters in the group's own order
        (reference `_get_zero_param_shapes`, `runtime/engine.py:3365-3400`: the order its ZeRO flattening uses)."""
        names = {id(p): n for n, p in self.module.named_parameters()}
        opt = self.optimizer
        if opt is not None and hasattr(opt, "param_to_og") and hasattr(opt, "opt_params"):
            groups = [OrderedDict() for _ in range(opt.num_og)]
            for p in opt.opt_params:
                if id(p) in names:
                    groups[opt.param_to_og[id(p)]][names[id(p)]] = torch.Size(getattr(p, "ds_shape", p.shape))
            return groups
        shapes = OrderedDict()
        for n, p in self.module.named_parameters():
            if p.requires_grad:
                shapes[n] = torch.Size(getattr(p, "ds_shape", p.shape))
        return [shapes]

    def _shared_params(self):
        """{alias name: canonical name} of tied parameters (reference `_get_shared_params`,
        `runtime/engine.py:3402-3430`): consolidation tools re-create the aliases from it."""
        first, shared = {}, {}
        for n, p in self.module.named_parameters(remove_duplicate=False):
            if id(p) in first:
                shared[n] = first[id(p)]
            else:
                first[id(p)] = n
        return shared

    def _checkpoint_tag_validation(self, tag):
        if not self._config.checkpoint_tag_validation_enabled or dist.get_world_size() == 1:
            return
        import hashlib
        b = hashlib.sha1(str(tag).encode()).digest()
        t = torch.tensor(list(b), dtype=torch.long, device=self.device)
        mx, mn = t.clone(), t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        ok = bool(torch.equal(mx, mn))
        if not ok:
            msg = f"[rank={dist.get_rank()}] The checkpoint tag name '{tag}' is not consistent across all ranks"
            if self._config.checkpoint_tag_validation_fail:
                raise ValueError(msg)
            logger.warning(msg)

    def _moe_layers(self):
        from ..moe.layer import MoE
        return [(n, m) for n, m in self.module.named_modules() if isinstance(m, MoE)]

    def _expert_ckpt_name(self, save_dir, tag, layer_id, expert_id):
        mp_rank = 0 if self.mpu is None else self.mpu.get_model_parallel_rank()
        return os.path.join(save_dir, str(tag), f"{CK.LAYER_FILE_PREFIX}{layer_id}_expert_{expert_id}_mp_rank_"
                            f"{mp_rank:02d}{CK.MODEL_FILE_SUFFIX}")

    def _save_moe_experts(self, save_dir, tag, module_sd):
        """One file per (MoE layer, GLOBAL expert id) with that expert's tensors (reference `_save_moe_checkpoint`,
        `runtime/engine.py:3151-3200`); written by expert-data-parallel rank 0 of each expert-parallel group. The
        expert entries are removed from `module_sd` (the main file holds only non-expert state)."""
        from ..checkpoint.zero_checkpoint import _EXPERT_RE
        for layer_id, (mname, m) in enumerate(self._moe_layers()):
            prefix = (mname + ".") if mname else ""
            keys = [k for k in list(module_sd.keys()) if k.startswith(prefix) and _EXPERT_RE.match(k)]
            per_expert = {}
            ep_rank = groups._get_expert_parallel_rank(m.expert_group_name) if dist.is_initialized() else 0
            edp_rank = groups._get_expert_data_parallel_rank(m.expert_group_name) if dist.is_initialized() else 0
            for k in keys:
                t = module_sd.pop(k)
                mm = _EXPERT_RE.match(k)
                gid = ep_rank * m.num_local_experts + int(mm.group(2))
                per_expert.setdefault(gid, OrderedDict())[f"{mm.group(1)}{gid}{mm.group(3)}"] = t.detach().clone()
            if edp_rank != 0:
                continue
            for gid, esd in per_expert.items():
                if all(t.numel() > 0 for t in esd.values()):  # ZeRO-3 placeholders live in the optimizer shards
                    self.checkpoint_engine.save(esd, self._expert_ckpt_name(save_dir, tag, layer_id, gid))

    def _load_moe_experts(self, load_dir, tag, module_sd):
        """Merge this rank's local experts from the per-expert files into `module_sd` (global -> local ids)."""
        from ..checkpoint.zero_checkpoint import _EXPERT_RE
        for layer_id, (mname, m) in enumerate(self._moe_layers()):
            ep_rank = groups._get_expert_parallel_rank(m.expert_group_name) if dist.is_initialized() else 0
            for local in range(m.num_local_experts):
                gid = ep_rank * m.num_local_experts + local
                path = self._expert_ckpt_name(load_dir, tag, layer_id, gid)
                if not os.path.exists(path):
                    continue
                esd = self.checkpoint_engine.load(path, map_location="cpu")
                for k, v in esd.items():
                    mm = _EXPERT_RE.match(k)
                    module_sd[f"{mm.group(1)}{local}{mm.group(3)}" if mm else k] = v

    def save_checkpoint(self, save_dir, tag=None, client_state={}, save_latest=True, exclude_frozen_parameters=False):
        """Reference layout (`runtime/engine.py:3050-3130`): `mp_rank_XX_model_states.pt` (ZeRO-3:
        `zero_pp_rank_{dp}_mp_rank_XX_model_states.pt` per rank, holding the partitioned placeholders), one
        `{bf16_}zero_pp_rank_{dp}_mp_rank_XX_optim_states.pt` per rank holding ONLY that rank's fp32 / moment shard
        plus the flat-layout descriptor, MoE expert files, `latest`, and `zero_to_fp32.py`. No rank gathers
        parameters it does not own."""
        if tag is None:
            tag = f"global_step{self.global_steps}"
        tag = str(tag)
        self._checkpoint_tag_validation(tag)
        if self._ckpt_lead_rank == 0:
            os.makedirs(os.path.join(save_dir, tag), exist_ok=True)
        dist.barrier()
        os.makedirs(os.path.join(save_dir, tag), exist_ok=True)
        self._curr_ckpt_path = os.path.join(save_dir, tag)
        module_sd = self.module_state_dict(exclude_frozen_parameters=exclude_frozen_parameters)
        if getattr(self, "has_moe_layers", False) and module_sd is not None:
            self._save_moe_experts(save_dir, tag, module_sd)
        zero = self.optimizer is not None
        sampler = None
        dl = getattr(self, "training_dataloader", None)
        if dl is not None and hasattr(getattr(dl, "data_sampler", None), "state_dict"):
            sampler = dl.data_sampler.state_dict()
        state = dict(module=module_sd if self.save_non_zero_checkpoint else None,
                     buffer_names=[n for n, _ in self.module.named_buffers()],
                     optimizer=None,
                     param_shapes=self._param_shapes() if zero else None,
                     frozen_param_shapes=None,
                     shared_params=self._shared_params(),
                     frozen_param_fragments=None,
                     lr_scheduler=self.lr_scheduler.state_dict() if self.lr_scheduler is not None else None,
                     data_sampler=sampler,
                     random_ltd=None,
                     sparse_tensor_module_names=list(self.sparse_tensor_module_names),
                     skipped_steps=self.skipped_steps,
                     global_steps=self.global_steps,
                     global_samples=self.global_samples,
                     dp_world_size=self.seq_dp_world_size,
                     mp_world_size=self.mp_world_size,
                     num_experts=getattr(self, "num_experts", None),
                     ds_config=self._config.param_dict,
                     ds_version=_version())
        state.update(client_state)
        if self.save_non_zero_checkpoint:
            self.checkpoint_engine.save(state, self._get_ckpt_name(save_dir, tag))
        if zero:
            osd = self.optimizer.state_dict(exclude_frozen_parameters=exclude_frozen_parameters)
            zsd = dict(optimizer_state_dict=osd, ds_config=self._config.param_dict, ds_version=_version())
            self.checkpoint_engine.save(zsd, self._get_zero_ckpt_name(save_dir, tag))
            if self._ckpt_lead_rank == 0:
                self._copy_recovery_script(save_dir)
        self.checkpoint_engine.commit(tag)
        dist.barrier()
        if zero and getattr(self._config.checkpoint_config, "write_reference_format", False):
            self._write_reference_format(save_dir, tag)
        if save_latest and self._ckpt_lead_rank == 0:
            with open(os.path.join(save_dir, "latest"), "w") as f:
                f.write(tag)
        dist.barrier()
        return True

    def _write_reference_format(self, save_dir, tag):
        """Every data-parallel rank re-slices the (complete, just committed) native shards into the file the
        reference would have written for it — no collective, one parameter in host memory at a time."""
        from ..checkpoint import reference_format as rf
        mp_rank = 0 if self.mpu is None else self.mpu.get_model_parallel_rank()
        rf.export_rank(save_dir, tag, dist.get_rank(self.seq_data_parallel_group),
                       dist.get_world_size(self.seq_data_parallel_group), mp_rank)
        dist.barrier()

    def _copy_recovery_script(self, save_path):
        import shutil
        src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "utils", "zero_to_fp32.py")
        if os.path.exists(src):
            shutil.copyfile(src, os.path.join(save_path, "zero_to_fp32.py"))

    def load_checkpoint(self, load_dir, tag=None, load_module_strict=True, load_optimizer_states=True,
                        load_lr_scheduler_states=True, load_module_only=False, custom_load_fn=None):
        """Reference `runtime/engine.py:2688-3020`. Optimizer state is restored positionally when this rank's saved
        flat layout equals the live one; otherwise (different data-parallel size, bucket size, persistence threshold,
        Twin-Flow ratio, or a reference-format checkpoint) every parameter's fp32 master AND Adam moments are
        rebuilt from all ranks' shards and re-partitioned (`checkpoint/zero_checkpoint.py`) — moments are never
        silently dropped."""
        from ..checkpoint import zero_checkpoint as zc
        if tag is None:
            latest = os.path.join(load_dir, "latest")
            if not os.path.isfile(latest):
                logger.warning(f"Unable to find latest file at {latest}")
                return None, None
            with open(latest) as f:
                tag = f.read().strip()
        tag_dir = os.path.join(load_dir, str(tag))
        path = self._get_ckpt_name(load_dir, tag)
        if not os.path.exists(path):
            # different topology: any model-states file carries the replicated metadata (and, outside ZeRO-3, the
            # full module)
            cands = sorted(f for f in os.listdir(tag_dir) if f.endswith(CK.MODEL_FILE_SUFFIX) and
                           not f.startswith(CK.LAYER_FILE_PREFIX))  # (layer_* = expert and pipeline-layer files)
            if not cands:
                raise FileNotFoundError(f"no model-states file in {tag_dir}")
            path = os.path.join(tag_dir, cands[0])
        ck = self.checkpoint_engine.load(path, map_location="cpu")
        module_sd = dict(ck.get("module") or {})
        self._curr_ckpt_path = tag_dir
        if getattr(self, "has_moe_layers", False):
            self._load_moe_experts(load_dir, tag, module_sd)
        placeholders = self._load_module_state(module_sd, strict=load_module_strict)
        universal = bool(self._config.checkpoint_config.get("load_universal", False)) \
            if isinstance(self._config.checkpoint_config, dict) else \
            bool(getattr(self._config.checkpoint_config, "load_universal", False))
        # under partitioned ZeRO-3 the weights themselves live in the optimizer shards
        # (also when THIS engine does not partition but the checkpoint was saved partitioned: placeholders)
        need_shards = self.optimizer is not None and (not load_module_only or self._zero3_partitioned() or
                                                      bool(placeholders))
        if universal and need_shards:
            from ..checkpoint.universal_checkpoint import load_universal_into
            tp_rank = 0 if self.mpu is None else self.mpu.get_model_parallel_rank()
            tp_size = 1 if self.mpu is None else self.mpu.get_model_parallel_world_size()
            load_universal_into(self.optimizer, self.module, tag_dir, tp_rank, tp_size)
        elif need_shards:
            with_states = load_optimizer_states and not load_module_only
            zpath = self._get_zero_ckpt_name(load_dir, tag)
            osd = None
            if os.path.exists(zpath):
                osd = self.checkpoint_engine.load(zpath, map_location="cpu")["optimizer_state_dict"]
            if osd is not None and CK.FLAT_LAYOUT in osd and \
                    zc.layouts_match(osd[CK.FLAT_LAYOUT], self.optimizer.layout()):
                # `load_from_fp32_weights: false` (reference `stage_1_and_2.py:2280-2310`): the masters are re-derived
                # from the 16-bit module weights of the checkpoint instead of its fp32 partitions; under ZeRO-3 the
                # module file holds placeholders, so the fp32 shards are the only source
                from_fp32 = bool(self._config.zero_config.load_from_fp32_weights) or self._zero3_partitioned()
                self.optimizer.load_state_dict(osd, load_optimizer_states=with_states, load_from_fp32_weights=from_fp32)
                if not from_fp32:
                    self.optimizer.refresh_from_module()
            elif zc.optim_files(tag_dir):
                src = zc.open_source(tag_dir, 0 if self.mpu is None else self.mpu.get_model_parallel_rank())
                log_dist(f"load_checkpoint: re-partitioning {type(src).__name__} ({len(src.files)} shard files) "
                         f"onto dp={self.optimizer.partition_count()}", ranks=[0])
                zc.restore_from_source(self.optimizer, self.module, src, load_optimizer_states=with_states)
                ref_osd = osd if osd is not None else zc.load_file(src.files[0])[CK.OPTIMIZER_STATE_DICT]
                self._load_scaler_state(ref_osd)
            else:
                self.optimizer.refresh_from_module()
        if load_lr_scheduler_states and self.lr_scheduler is not None and ck.get("lr_scheduler") is not None:
            self.lr_scheduler.load_state_dict(ck["lr_scheduler"])
        dl = getattr(self, "training_dataloader", None)
        if ck.get("data_sampler") is not None and dl is not None and hasattr(getattr(dl, "data_sampler", None),
                                                                             "load_state_dict"):
            dl.data_sampler.load_state_dict(ck["data_sampler"])
        self.global_steps = ck.get("global_steps", 0)
        self.global_samples = ck.get("global_samples", self.global_steps * self.train_batch_size())
        self.skipped_steps = ck.get("skipped_steps", 0)
        client_state = {k: v for k, v in ck.items() if k not in _CKPT_KEYS}
        return tag_dir, client_state

    def _load_scaler_state(self, osd):
        opt = self.optimizer
        ls = osd.get(CK.LOSS_SCALER)
        if isinstance(ls, dict):
            opt.loss_scaler.load_state_dict(ls)
        elif ls is not None and hasattr(ls, "cur_scale"):  # reference LossScaler object (stubbed on load)
            opt.loss_scaler.cur_scale = float(getattr(ls, "cur_scale"))
        opt.dynamic_loss_scale = osd.get("dynamic_loss_scale", opt.dynamic_loss_scale)

    @torch.no_grad()
    def _load_module_state(self, sd, strict=True):
        """Load a module state dict. Under ZeRO-3 the dict of a partitioned run holds empty placeholders for the
        partitioned parameters (their values live in the optimizer shards): those names are returned so the caller
        restores them from the shards; real shape mismatches and (with `strict`) missing keys raise."""
        if self.zero_optimization_partition_weights() and self.optimizer is not None:
            own = dict(self.module.named_parameters())
            placeholders, bad = [], []
            wrote = False
            for n, v in sd.items():
                p = own.get(n)
                if p is None or not torch.is_tensor(v):
                    continue
                want = getattr(p, "ds_numel", p.numel())
                if v.numel() == want and v.numel() > 0:
                    if id(p) not in self.optimizer.param_group:  # kept whole on every rank (small / other dtype)
                        p.data.copy_(v.reshape(p.shape))
                        continue
                    # local copy into this rank's partition; the full buffers are refreshed once below
                    self.optimizer._scatter_param(p, v, "fp32", also_shard=True)
                    wrote = True
                elif v.numel() == 0 and want > 0:
                    placeholders.append(n)
                else:
                    bad.append(f"{n}: checkpoint {tuple(v.shape)} vs model {tuple(getattr(p, 'ds_shape', p.shape))}")
            if bad:
                raise RuntimeError("size mismatch loading module state: " + "; ".join(bad[:5]))
            if strict:
                missing = [n for n in own if n not in sd]
                if missing:
                    raise RuntimeError(f"missing keys in checkpoint module state: {missing[:5]}")
            if wrote:
                self.optimizer._post_step_gather()
            bufs = dict(self.module.named_buffers())
            for n, v in sd.items():
                if n in bufs:
                    bufs[n].copy_(v)
            return placeholders
        self.module.load_state_dict(sd, strict=strict)
        if self.optimizer is not None:
            self.optimizer.refresh_from_module()
        return []


    # ============================================================================================ small API surface
    def destroy(self):
        """Drop the hooks and buffers the engine hung on the module (reference `runtime/engine.py:369-373`)."""
        opt = self.optimizer
        if opt is not None:
            opt.join_offload()
            if getattr(opt, "coordinator", None) is not None:
                opt.coordinator.remove_hooks()
            for h in getattr(opt, "_hooks", []):
                h.remove()
            opt._hooks = []
        if self.checkpoint_engine is not None:
            self.checkpoint_engine.commit("destroy")

    def was_step_applied(self) -> bool:
        """False when the last `step()` fell inside an accumulation window or was skipped for overflow (reference
        `runtime/engine.py:1300-1309`)."""
        return bool(getattr(self, "_step_applied", False))

    def get_batch_info(self):
        """(train_batch_size, train_micro_batch_size_per_gpu, gradient_accumulation_steps)."""
        return self.train_batch_size(), self.train_micro_batch_size_per_gpu(), self.gradient_accumulation_steps()

    def set_train_micro_batch_size(self, micro_batch_size):
        """New micro-batch size at the same accumulation depth (reference `runtime/engine.py:446-452`)."""
        gas = self.gradient_accumulation_steps()
        self._config.train_batch_size = micro_batch_size * gas * self.dp_world_size
        self._config.train_micro_batch_size_per_gpu = micro_batch_size

    def get_type(self):
        """Optimizer hyper-parameter "type" per param group (reference `runtime/engine.py:1823`)."""
        return [g.get("type") for g in self.optimizer.param_groups] if self.optimizer is not None else None

    def get_data_types(self):
        """(model dtype, gradient-accumulation dtype), reference `runtime/engine.py:1031-1044`."""
        model_dtype = self._dtype()
        acc = self._config.grad_accum_dtype
        acc_dtype = {None: None, "fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}.get(acc)
        if acc_dtype is None:
            acc_dtype = torch.float32 if model_dtype == torch.bfloat16 else model_dtype
        return model_dtype, acc_dtype

    def dynamic_loss_scale(self):
        return self._config.loss_scale == 0

    def postscale_gradients(self):
        return not self._config.prescale_gradients

    def zero_cpu_offload(self):
        return self.zero_offload_optimizer() is not None and \
            str(getattr(self.zero_offload_optimizer().device, "value", self.zero_offload_optimizer().device)) == "cpu"

    zero_use_cpu_optimizer = zero_cpu_offload

    def zero_has_nvme_offload(self):
        devs = [getattr(o, "device", None) for o in (self.zero_offload_optimizer(), self.zero_offload_param())
                if o is not None]
        return any(str(getattr(d, "value", d)) == "nvme" for d in devs)

    def zero_partial_offload(self):
        o = self.zero_offload_optimizer()
        return float(getattr(o, "ratio", 1.0)) if o is not None else 1.0

    def get_pld_theta(self):
        return self.progressive_layer_drop.get_theta() if self.progressive_layer_drop is not None else None

    def pld_theta(self):
        return self._config.pld_params.get("theta", 1.0) if self._config.pld_params else None

    def pld_gamma(self):
        return self._config.pld_params.get("gamma", 0.001) if self._config.pld_params else None

    def random_ltd_enabled(self):
        de = self._config.data_efficiency_config or {}
        return bool(de.get("enabled", False) and de.get("data_routing", {}).get("random_ltd", {}).get("enabled", False))

    def random_ltd_config(self):
        return (self._config.data_efficiency_config or {}).get("data_routing", {}).get("random_ltd", {})

    def data_sampling_enabled(self):
        de = self._config.data_efficiency_config or {}
        return bool(de.get("enabled", False) and de.get("data_sampling", {}).get("enabled", False))

    def data_sampling_config(self):
        return (self._config.data_efficiency_config or {}).get("data_sampling", {})

    def curriculum_learning_config(self):
        return self.data_sampling_config().get("curriculum_learning", {})

    def set_custom_curriculum_learning_schedule(self, schedule_func_dict):
        """Install client difficulty schedules (reference `runtime/engine.py:1742-1744`): {metric: fn(step)}."""
        dl = self.training_dataloader
        sampler = getattr(dl, "data_sampler", None)
        if sampler is None or not hasattr(sampler, "set_custom_curriculum_learning_schedule"):
            raise RuntimeError("no curriculum data sampler: enable data_efficiency.data_sampling.curriculum_learning "
                               "and build the loader with engine.deepspeed_io")
        sampler.set_custom_curriculum_learning_schedule(schedule_func_dict)

    def flops_profiler_enabled(self):
        return self._config.flops_profiler_config.enabled

    def flops_profiler_profile_step(self):
        return self._config.flops_profiler_config.profile_step

    def flops_profiler_module_depth(self):
        return self._config.flops_profiler_config.module_depth

    def flops_profiler_top_modules(self):
        return self._config.flops_profiler_config.top_modules

    def flops_profiler_detailed(self):
        return self._config.flops_profiler_config.detailed

    def flops_profiler_output_file(self):
        return self._config.flops_profiler_config.output_file

    def autotuning_enabled(self):
        return bool((self._config.autotuning_config or {}).get("enabled", False))

    def autotuning_metric(self):
        return (self._config.autotuning_config or {}).get("metric", "throughput")

    def autotuning_metric_path(self):
        return (self._config.autotuning_config or {}).get("metric_path")

    def autotuning_start_profile_step(self):
        return (self._config.autotuning_config or {}).get("start_profile_step", 3)

    def autotuning_end_profile_step(self):
        return (self._config.autotuning_config or {}).get("end_profile_step", 5)

    @staticmethod
    def is_map_style_dataset(obj):
        return hasattr(obj, "__getitem__") and hasattr(obj, "__len__")

    @staticmethod
    def is_iterable_style_dataset(obj):
        return isinstance(obj, torch.utils.data.IterableDataset)

    def empty_partition_cache(self):
        """Release every gathered ZeRO-3 parameter now (reference `runtime/engine.py:3594-3602`), e.g. between an
        evaluation pass and the next training step."""
        coord = getattr(self.optimizer, "coordinator", None) if self.optimizer is not None else None
        if coord is not None:
            for g in self.optimizer.all_groups:
                if not g.persistent:
                    coord.release(g)
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def load_module_state_dict(self, checkpoint=None, strict=True, custom_load_fn=None, fetch_z3_params=False):
        """Load module weights from a loaded checkpoint dict (its "module" entry) or a plain state dict (reference
        `runtime/engine.py:2553-2590`); the optimizer's master weights follow the loaded values."""
        sd = checkpoint.get("module", checkpoint) if isinstance(checkpoint, dict) else checkpoint
        if custom_load_fn is not None:
            custom_load_fn(src=sd, dst=self.module)
            if self.optimizer is not None and not self._zero3_partitioned():
                self.optimizer.refresh_from_module()
            return []
        return self._load_module_state(dict(sd or {}), strict=strict)

    def update_optimizer_step(self, step):
        """Overwrite the optimizer's step counter (reference `runtime/engine.py:2600-2614`)."""
        if hasattr(self.optimizer, "set_step"):
            self.optimizer.set_step(step)
        else:
            for st in self.optimizer.state.values():
                if "step" in st:
                    st["step"] = step

    def print_forward_breakdown(self, fwd_time):
        """MoE time split of the forward pass (reference `runtime/engine.py:1776-1796`)."""
        gate = moe = falltoall = salltoall = 0.0
        for _, m in self._moe_layers():
            layer = m.deepspeed_moe
            gate += getattr(layer.gate, "gate_time", 0.0)
            moe += layer.time_moe
            falltoall += layer.time_falltoall
            salltoall += layer.time_salltoall
        log_dist(f"time (ms) | fwd: {fwd_time:.2f} (fwd_moe: {moe:.2f}, 1st_a2a: {falltoall:.2f}, "
                 f"2nd_a2a: {salltoall:.2f}, top_k: {gate:.2f})", ranks=[0])


    def save_16bit_model(self, save_dir, save_filename="pytorch_model.bin", exclude_frozen_parameters=False):
        """Consolidated 16-bit weights, streamed group by group to rank 0 (reference `runtime/engine.py:3477`). As in
        the reference (`engine.py:3618-3626`) a ZeRO-3 partitioned model is only gathered when
        `stage3_gather_16bit_weights_on_model_save` allows it."""
        if self._zero3_partitioned() and not self._config.zero_config.gather_16bit_weights_on_model_save:
            logger.info(f"Did not save the model {os.path.join(save_dir, save_filename)} because "
                        "`stage3_gather_16bit_weights_on_model_save` is False")
            return False
        sd = self.consolidated_16bit_state_dict(exclude_frozen_parameters=exclude_frozen_parameters)
        if dist.get_rank() == 0:
            os.makedirs(save_dir, exist_ok=True)
            torch.save(sd, os.path.join(save_dir, save_filename))
        dist.barrier()
        return True

    save_fp16_model = save_16bit_model



# ------------------------------------------------------------------------------------------------ accessor surface
# The reference engine exposes most configuration values as zero-argument methods (`runtime/engine.py:470-880`);
# client code and integrations (HF Trainer, Megatron-DeepSpeed) call them. They are generated from two tables:
# method name -> attribute of the parsed config, and method name -> field of the ZeRO sub-config.
_CONFIG_ACCESSORS = {
    "dump_state": "dump_state", "optimizer_name": "optimizer_name", "optimizer_params": "optimizer_params",
    "optimizer_legacy_fusion": "optimizer_legacy_fusion", "scheduler_name": "scheduler_name",
    "scheduler_params": "scheduler_params", "amp_params": "amp_params", "aio_config": "aio_config",
    "dynamic_loss_scale_args": "dynamic_loss_scale_args", "initial_dynamic_scale": "initial_dynamic_scale",
    "gradient_predivide_factor": "gradient_predivide_factor", "sparse_gradients_enabled": "sparse_gradients_enabled",
    "communication_data_type": "communication_data_type", "dataloader_drop_last": "dataloader_drop_last",
    "elasticity_enabled": "elasticity_enabled", "pld_enabled": "pld_enabled", "pld_params": "pld_params",
    "curriculum_enabled_legacy": "curriculum_enabled_legacy", "curriculum_params_legacy": "curriculum_params_legacy",
    "data_efficiency_enabled": "data_efficiency_enabled", "data_efficiency_config": "data_efficiency_config",
    "eigenvalue_enabled": "eigenvalue_enabled", "eigenvalue_verbose": "eigenvalue_verbose",
    "eigenvalue_max_iter": "eigenvalue_max_iter", "eigenvalue_tol": "eigenvalue_tol",
    "eigenvalue_stability": "eigenvalue_stability", "eigenvalue_layer_name": "eigenvalue_layer_name",
    "eigenvalue_layer_num": "eigenvalue_layer_num",
    "eigenvalue_gas_boundary_resolution": "eigenvalue_gas_boundary_resolution",
    "checkpoint_tag_validation_enabled": "checkpoint_tag_validation_enabled",
    "checkpoint_tag_validation_fail": "checkpoint_tag_validation_fail",
    "load_universal_checkpoint": "load_universal_checkpoint", "use_node_local_storage": "use_node_local_storage",
    "graph_harvesting": "graph_harvesting", "fp16_auto_cast": "fp16_auto_cast",
    "fp16_master_weights_and_gradients": "fp16_master_weights_and_gradients",
    "zero_allow_untested_optimizer": "zero_allow_untested_optimizer",
    "zero_force_ds_cpu_optimizer": "zero_force_ds_cpu_optimizer", "mics_shard_size": "mics_shard_size",
    "swap_tensor_config": "aio_config",
}
_ZERO_ACCESSORS = {
    "zero_reduce_scatter": "reduce_scatter", "zero_overlap_comm": "overlap_comm",
    "zero_contiguous_gradients": "contiguous_gradients", "zero_reduce_bucket_size": "reduce_bucket_size",
    "zero_multi_rank_bucket_allreduce": "use_multi_rank_bucket_allreduce",
    "zero_allgather_bucket_size": "allgather_bucket_size", "zero_allgather_partitions": "allgather_partitions",
    "zero_sub_group_size": "sub_group_size", "zero_prefetch_bucket_size": "prefetch_bucket_size",
    "zero_param_persistence_threshold": "param_persistence_threshold",
    "zero_model_persistence_threshold": "model_persistence_threshold",
    "zero_max_live_parameters": "max_live_parameters", "zero_max_reuse_distance": "max_reuse_distance",
    "zero_gather_16bit_weights_on_model_save": "gather_16bit_weights_on_model_save",
    "zero_ignore_unused_parameters": "ignore_unused_parameters", "zero_legacy_stage1": "legacy_stage1", "zero_grad_hooks": "grad_hooks",
    "zero_round_robin_gradients": "round_robin_gradients", "zero_load_from_fp32_weights": "load_from_fp32_weights",
    "zero_elastic_checkpoint": "elastic_checkpoint", "zero_hpz_partition_size": "zero_hpz_partition_size",
    "zero_quantized_weights": "zero_quantized_weights", "zero_quantized_gradients": "zero_quantized_gradients",
    "zero_quantized_nontrainable_weights": "zero_quantized_nontrainable_weights",
}


def _install_accessors():
    def cfg_getter(attr):
        return lambda self: getattr(self._config, attr)

    def zero_getter(attr):
        return lambda self: getattr(self._config.zero_config, attr)

    for name, attr in _CONFIG_ACCESSORS.items():
        if name not in DeepSpeedEngine.__dict__:
            setattr(DeepSpeedEngine, name, cfg_getter(attr))
    for name, attr in _ZERO_ACCESSORS.items():
        if name not in DeepSpeedEngine.__dict__:
            setattr(DeepSpeedEngine, name, zero_getter(attr))


_install_accessors()

_CKPT_KEYS = {
    "module", "buffer_names", "optimizer", "param_shapes", "frozen_param_shapes", "shared_params",
    "frozen_param_fragments", "lr_scheduler", "data_sampler", "random_ltd", "sparse_tensor_module_names",
    "skipped_steps", "global_steps", "global_samples", "dp_world_size", "mp_world_size", "ds_config", "ds_version",
    "num_experts"
}
