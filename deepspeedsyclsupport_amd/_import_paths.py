"""Reference import paths that have no file of their own here.

This framework folds several reference modules into one (one flat ZeRO optimizer instead of `stage_1_and_2.py` /
`stage3.py` / `bf16_optimizer.py` / `fp16/fused_optimizer.py`, one monitor module, one accelerator module, ...).
Client code written against the reference imports those paths, so a meta-path finder serves them: every entry of
`PATHS` names the module that really holds the code and the reference names it should be visible under. Nothing is
imported until a client asks for the path.
"""
import importlib
import importlib.abc
import importlib.machinery
import sys
import types

_PKG = __name__.rsplit(".", 1)[0]

# reference path (below the package) -> [(real module (below the package), {exposed name: real name} or "*")]
PATHS = {
    "runtime.zero.stage3": [("runtime.zero.flat_optimizer", {"DeepSpeedZeroOptimizer_Stage3": "DeepSpeedZeroOptimizer_Stage3",
                                                            "estimate_zero3_model_states_mem_needs": "estimate_zero3_model_states_mem_needs", "estimate_zero3_model_states_mem_needs_all_live": "estimate_zero3_model_states_mem_needs_all_live", "estimate_zero3_model_states_mem_needs_all_cold": "estimate_zero3_model_states_mem_needs_all_cold", "model_to_params": "model_to_params"})],
    "runtime.zero.stage_1_and_2": [("runtime.zero.flat_optimizer", {"DeepSpeedZeroOptimizer": "DeepSpeedZeroOptimizer",
                                                                   "estimate_zero2_model_states_mem_needs": "estimate_zero2_model_states_mem_needs", "estimate_zero2_model_states_mem_needs_all_live": "estimate_zero2_model_states_mem_needs_all_live", "estimate_zero2_model_states_mem_needs_all_cold": "estimate_zero2_model_states_mem_needs_all_cold", "model_to_params": "model_to_params"})],
    "runtime.zero.partitioned_param_coordinator": [("runtime.zero.coordinator",
                                                    {"PartitionedParameterCoordinator": "ParamCoordinator",
                                                     "ZeRoTraceMode": "ZeRoTraceMode",
                                                     "InflightParamRegistry": "InflightParamRegistry",
                                                     "iter_params": "iter_params",
                                                     "get_all_parameters": "get_all_parameters"})],
    "runtime.zero.parameter_offload": [("runtime.zero.coordinator", {"DeepSpeedZeRoOffload": "ParamCoordinator"})],
    "runtime.zero.mics": [("runtime.zero", {"MiCS_Init": "MiCS_Init", "MiCS_Optimizer": "MiCS_Optimizer"}),
                          ("runtime.zero.mics_utils", {"MiCS_CommGroups": "MiCS_CommGroups",
                                                       "create_mics_comm_groups": "create_mics_comm_groups"})],
    "runtime.bf16_optimizer": [("runtime.zero.flat_optimizer", {"BF16_Optimizer": "BF16_Optimizer"})],
    "runtime.fp16.fused_optimizer": [("runtime.zero.flat_optimizer", {"FP16_Optimizer": "FP16_Optimizer"})],
    "runtime.fp16.unfused_optimizer": [("runtime.zero.flat_optimizer", {"FP16_UnfusedOptimizer": "FP16_Optimizer"})],
    "runtime.constants": [("runtime.config", "*")],
    "module_inject.load_checkpoint": [("runtime.state_dict_factory", {"load_model_with_checkpoint": "load_hf_shards"})],
    "module_inject.module_quantize": [("runtime.weight_quantizer", "*")],
    "monitor.config": [("runtime.config", {"DeepSpeedMonitorConfig": "MonitorConfig", "TensorBoardConfig": "TensorBoardConfig",
                                           "WandbConfig": "WandbConfig", "CSVConfig": "CSVConfig"})],
    "monitor.tensorboard": [("monitor.monitor", {"TensorBoardMonitor": "TensorBoardMonitor"})],
    "monitor.wandb": [("monitor.monitor", {"WandbMonitor": "WandbMonitor"})],
    "monitor.csv_monitor": [("monitor.monitor", {"csvMonitor": "csvMonitor"})],
    "profiling.config": [("runtime.config", {"DeepSpeedFlopsProfilerConfig": "FlopsProfilerConfig"})],
    "comm.config": [("runtime.config", {"DeepSpeedCommsConfig": "CommsLoggerConfig", "CommsLoggerConfig": "CommsLoggerConfig"})],
    "comm.utils": [("comm.comm", "*")],
    "comm.torch": [("comm.comm", "*")],
    "accelerator.real_accelerator": [("accelerator", {"get_accelerator": "get_accelerator",
                                                      "set_accelerator": "set_accelerator"})],
    "constants": [("comm.comm", {"TORCH_DISTRIBUTED_DEFAULT_PORT": "TORCH_DISTRIBUTED_DEFAULT_PORT",
                                 "default_pg_timeout": "default_pg_timeout"})],
    "pydantic_v1": [("runtime.config_utils", "*")],
    # ---- training runtime
    "runtime.activation_checkpointing.config": [("runtime.config", {"DeepSpeedActivationCheckpointingConfig":
                                                                    "ActivationCheckpointingConfig"})],
    "runtime.checkpoint_engine.torch_checkpoint_engine": [("runtime.checkpoint_engine.checkpoint_engine",
                                                           {"TorchCheckpointEngine": "TorchCheckpointEngine"})],
    "runtime.checkpoint_engine.nebula_checkpoint_engine": [("runtime.checkpoint_engine.checkpoint_engine",
                                                            {"NebulaCheckpointEngine": "AsyncCheckpointEngine"})],
    "runtime.comm.nccl": [("runtime.comm.compressed", {"NcclBackend": "CompressedBackend"})],
    "runtime.comm.mpi": [("runtime.comm.compressed", {"MpiBackend": "CompressedBackend"})],
    "runtime.comm.hccl": [("runtime.comm.compressed", {"HcclBackend": "CompressedBackend"})],
    "runtime.compression.cupy": [("runtime.comm.compressed", {"pack_signs": "pack_signs",
                                                              "unpack_signs": "unpack_signs"})],
    "runtime.swap_tensor.async_swapper": [("runtime.swap_tensor.tensor_swapper",
                                           {"AsyncTensorSwapper": "AsyncTensorSwapper"})],
    "runtime.swap_tensor.partitioned_optimizer_swapper": [("runtime.swap_tensor.optimizer_swapper",
                                                           {"PartitionedOptimizerSwapper": "OptimizerStateSwapper"})],
    "runtime.swap_tensor.pipelined_optimizer_swapper": [("runtime.swap_tensor.optimizer_swapper",
                                                         {"PipelinedOptimizerSwapper": "OptimizerStateSwapper"})],
    "runtime.swap_tensor.optimizer_utils": [("runtime.swap_tensor.optimizer_swapper",
                                             {"OptimizerSwapper": "OptimizerStateSwapper", "NvmeFlat": "NvmeFlat"})],
    "runtime.swap_tensor.partitioned_param_swapper": [("runtime.swap_tensor.param_store",
                                                       {"AsyncPartitionedParameterSwapper": "ParamNvmeStore"})],
    "runtime.swap_tensor.aio_config": [("runtime.config", {"AIOConfig": "AIOConfig"})],
    "runtime.data_pipeline.config": [("runtime.config", {"DeepSpeedConfig": "DeepSpeedConfig"})],
    "runtime.data_pipeline.data_routing.helper": [("runtime.data_pipeline.data_routing.basic_layer",
                                                   {"convert_to_random_ltd": "convert_to_random_ltd"})],
    "runtime.data_pipeline.data_routing.utils": [("ops.random_ltd", "*")],
    "runtime.data_pipeline.data_sampling.utils": [("runtime.data_pipeline.data_sampling.indexed_dataset", "*"),
                                                  ("runtime.data_pipeline.data_sampling.data_analyzer",
                                                   {"split_index": "split_index", "split_dataset": "split_dataset"})],
    "autotuning.scheduler": [("autotuning.autotuner", {"ResourceManager": "ResourceManager"})],
    "monitor.utils": [("monitor.monitor", {"check_tb_availability": "check_tb_availability",
                                           "check_wandb_availability": "check_wandb_availability"})],
    # ---- ops
    "ops.deepspeed4science.evoformer_attn": [("ops.deepspeed4science", "*")],
    "ops.random_ltd.dropping_utils": [("ops.random_ltd", "*")],
    "ops.sparse_attention.bert_sparse_self_attention": [("ops.sparse_attention.sparse_self_attention",
                                                         {"BertSparseSelfAttention": "BertSparseSelfAttention"})],
    "ops.sparse_attention.sparse_attention_utils": [("ops.sparse_attention.sparse_self_attention",
                                                     {"SparseAttentionUtils": "SparseAttentionUtils"})],
    "ops.transformer.inference.ds_mlp": [("ops.transformer.inference.ds_attention", {"DeepSpeedMLP": "DeepSpeedMLP"})],
    **{f"ops.transformer.inference.op_binding.{f}": [("ops.transformer.inference.op_binding", {n: n, "BaseOp": "BaseOp"})]
       for f, n in (("base", "BaseOp"), ("gelu_gemm", "GELUGemmOp"), ("linear", "LinearOp"), ("mlp_gemm", "MLPGemmOp"),
                    ("qkv_gemm", "QKVGemmOp"), ("residual_add", "ResidualAddOp"), ("softmax", "SoftmaxOp"),
                    ("softmax_context", "SoftmaxContextOp"), ("vector_matmul", "VectorMatMulOp"))},
    "ops.transformer.inference.bias_add": [("ops.spatial", {"nhwc_bias_add": "nhwc_bias_add"})],
    "ops.transformer.inference.moe_inference": [
        ("ops.transformer.inference.layer", {"DeepSpeedMoEInference": "DeepSpeedMoEInference"}),
        ("ops.transformer.inference.config", {"DeepSpeedMoEInferenceConfig": "DeepSpeedMoEInferenceConfig"})],
    "ops.transformer.inference.diffusers_2d_transformer": [
        ("module_inject.diffusers", {"Diffusers2DTransformerConfig": "Diffusers2DTransformerConfig"})],
    "ops.transformer.inference.diffusers_attention": [("module_inject.diffusers",
                                                       {"DeepSpeedDiffusersAttention": "DSDiffusersAttention"})],
    "ops.transformer.inference.diffusers_transformer_block": [
        ("module_inject.diffusers", {"DeepSpeedDiffusersTransformerBlock": "DSDiffusersTransformerBlock"})],
    **{f"module_inject.containers.{f}": [("module_inject.containers", "*")]
       for f in ("base", "base_moe", "bert", "bloom", "clip", "distil_bert", "gpt2", "gptj", "gptneo", "gptneox",
                 "internlm", "llama", "llama2", "megatron_gpt", "megatron_gpt_moe", "opt", "unet", "vae")},
    **{f"module_inject.containers.features.{f}": [("module_inject.container_features", "*")]
       for f in ("gated_mlp", "hybrid_engine", "hybrid_megatron", "megatron", "meta_tensor", "split_qkv")},
    "module_inject.containers.features": [("module_inject.container_features", "*")],
    "module_inject.replace_policy": [("module_inject.containers", {"replace_policies": "replace_policies",
                                                                  "generic_policies": "generic_policies"})],
    "module_inject.utils": [("module_inject.containers", {"policy_to_ds_container": "policy_to_ds_container"})],
    "module_inject.inject": [("module_inject.containers", {"module_inject": "replace_layers_with_policy"})],
    # ---- inference v1 model wrappers: one fused layer serves every architecture
    "model_implementations.diffusers.unet": [("module_inject.diffusers", {"DSUNet": "DSUNet"})],
    "model_implementations.diffusers.vae": [("module_inject.diffusers", {"DSVAE": "DSVAE"})],
    "model_implementations.transformers.clip_encoder": [("module_inject.diffusers",
                                                         {"DSClipEncoder": "DSClipEncoder"})],
    "model_implementations.features.cuda_graph": [("module_inject.diffusers", {"CUDAGraph": "GraphedCall"})],
    "model_implementations.transformers.ds_transformer": [
        ("ops.transformer.inference.layer", {"DeepSpeedTransformerInference": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_base": [
        ("ops.transformer.inference.layer", {"DeepSpeedTransformerBase": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_bert": [
        ("ops.transformer.inference.layer", {"DeepSpeedBERTInference": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_bloom": [
        ("ops.transformer.inference.layer", {"DeepSpeedBloomInference": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_gpt": [
        ("ops.transformer.inference.layer", {"DeepSpeedGPTInference": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_llama2": [
        ("ops.transformer.inference.layer", {"DeepSpeedLlama2Inference": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_megatron_gpt": [
        ("ops.transformer.inference.layer", {"DeepSpeedMegatronGPTInference": "DeepSpeedTransformerInference"})],
    "model_implementations.transformers.ds_opt": [
        ("ops.transformer.inference.layer", {"DeepSpeedOPTInference": "DeepSpeedTransformerInference"})],
    # ---- inference v2: the reference's one-class-per-file tree over this package's per-family modules
    "inference.v2.ragged.blocked_allocator": [("inference.kv_cache", {"BlockedAllocator": "BlockedAllocator"})],
    "inference.v2.ragged.kv_cache": [("inference.kv_cache", {"BlockedKVCache": "BlockedKVCache",
                                                             "split_kv": "split_kv"})],
    "inference.v2.ragged.manager_configs": [("inference.v2.config_v2", "*")],
    **{f"inference.v2.kernels.core_ops.{d}.{f}": [("inference.v2.kernels.core_ops", {n: n for n in names})]
       for d, f, names in (
           ("bias_activations", "bias_activation", ("CUDABiasActivation", )),
           ("blas_kernels", "blas_linear", ("BlasLibLinear", )),
           ("cuda_layer_norm", "cuda_fp_ln_base", ("CUDAFPLNBase", )),
           ("cuda_layer_norm", "cuda_ln", ("CUDAFPLN", )),
           ("cuda_layer_norm", "cuda_post_ln", ("CUDAFPPostLN", )),
           ("cuda_layer_norm", "cuda_pre_ln", ("CUDAFPPreLN", )),
           ("cuda_rms_norm", "rms_norm_base", ("CUDARMSNormBase", )),
           ("cuda_rms_norm", "rms_norm", ("CUDARMSNorm", )),
           ("cuda_rms_norm", "rms_pre_norm", ("CUDARMSPreNorm", )),
           ("gated_activations", "gated_activation", ("CUDAGatedActivation", )))},
    **{f"inference.v2.kernels.cutlass_ops.{d}.{f}": [("inference.v2.kernels.cutlass_ops", {n: n})]
       for d, f, n in (("mixed_gemm", "mixed_gemm", "MixedGEMM"), ("moe_gemm", "moe_gemm", "MoEGEMM"),
                       ("moe_gemm", "mixed_moe_gemm", "MixedMoEGEMM"))},
    **{f"inference.v2.kernels.ragged_ops.{d}.{f}": [("inference.v2.kernels.ragged_ops", {n: n for n in names})]
       for d, f, names in (
           ("atom_builder", "atom_builder", ("AtomBuilder", )),
           ("blocked_flash", "blocked_flash", ("BlockedFlashAttn", "get_q_block_size", "get_kv_block_size")),
           ("embed", "embed", ("RaggedEmbeddingKernel", )),
           ("linear_blocked_kv_rotary", "blocked_kv_rotary", ("BlockedRotaryEmbeddings", )),
           ("linear_blocked_kv_rotary", "blocked_trained_kv_rotary", ("BlockedTrainedRotaryEmbeddings", )),
           ("linear_blocked_kv_rotary", "linear_blocked_kv_copy", ("LinearBlockedKVCopy", )),
           ("logits_gather", "logits_gather", ("RaggedLogitsGather", )),
           ("moe_gather", "moe_gather", ("MoEGather", )),
           ("moe_scatter", "moe_scatter", ("MoEScatter", )),
           ("top_k_gating", "top_k_gating", ("RaggedTopKGating", )))},
    **{f"inference.v2.modules.configs.{f}": [("inference.v2.modules.configs", "*")]
       for f in ("attention_configs", "embedding_config", "linear_config", "moe_config", "norm_config",
                 "unembed_config")},
    **{f"inference.v2.modules.interfaces.{f}": [("inference.v2.modules.interfaces", "*")]
       for f in ("attention_base", "embedding_base", "linear_base", "moe_base", "post_norm_base", "pre_norm_base",
                 "unembed_base")},
    **{f"inference.v2.modules.implementations.{d}.{f}": [("inference.v2.modules.implementations", {n: n})]
       for d, f, n in (("attention", "dense_blocked_attention", "DSDenseBlockedAttention"),
                       ("embedding", "ragged_embedding", "DSRaggedEmbedding"),
                       ("linear", "blas_fp_linear", "BlasFPLinear"),
                       ("moe", "cutlass_multi_gemm", "DSMultiGemmMoE"),
                       ("post_norm", "cuda_post_ln", "DSPostLNCUDAModule"),
                       ("pre_norm", "cuda_pre_ln", "DSPreLNCUDAModule"),
                       ("pre_norm", "cuda_pre_rms", "DSPreRMSCUDAModule"),
                       ("unembed", "ragged_unembed", "DSRaggedUnembed"))},
    **{f"inference.v2.model_implementations.common_parameters.{f}": [
        ("inference.v2.model_implementations.common_parameters", "*")]
       for f in ("attn_output_parameters", "embedding_parameters", "invfreq_parameters", "mlp_parameters",
                 "moe_parameters", "norm_parameters", "qkv_parameters", "unembed_parameters")},
    **{f"inference.v2.model_implementations.sharding.{f}": [("inference.v2.model_implementations.sharding", "*")]
       for f in ("attn", "attn_out", "embedding", "mlp", "qkv", "types", "unembed", "utils")},
    **{f"inference.v2.model_implementations.{a}.{f}": [("inference.v2.model_implementations.archs", "*")]
       for a in ("llama_v2", "mistral", "mixtral", "opt", "phi", "falcon")
       for f in ("container", "containers", "model", "policy")},
}
# (File modules of this package that sub-paths hang under — `core_ops.py`, `ragged_ops.py`, `configs.py`, ... — carry
# `__path__ = []`, so the import system asks the finder for their "submodules".)



def _section_constants(section, model_path, model_name, prefix=None, extra=None):
    """Names the reference's `constants.py` files define for a config section, derived from the pydantic model that
    parses it here: SECTION = "section", SECTION_KEY = "key", SECTION_KEY_DEFAULT = default."""

    def build():
        model = getattr(importlib.import_module(f"{_PKG}.{model_path}"), model_name)
        pre = (prefix or section).upper()
        out = {pre: section, f"{pre}_FORMAT": f'"{section}": {{...}}'}
        for key, field in model.model_fields.items():
            out[f"{pre}_{key.upper()}"] = key
            if not field.is_required():
                out[f"{pre}_{key.upper()}_DEFAULT"] = field.get_default(call_default_factory=True)
        out.update(extra or {})
        return out

    return build


# reference path -> callable returning the module's names
GENERATED = {
    "comm.constants": _section_constants("comms_logger", "runtime.config", "CommsLoggerConfig", extra={
        "NCCL_BACKEND": "nccl", "CCL_BACKEND": "ccl", "MPI_BACKEND": "mpi", "GLOO_BACKEND": "gloo",
        "SCCL_BACKEND": "sccl", "HCCL_BACKEND": "hccl", "DEFAULT_AML_MASTER_PORT": "54965",
        "DEFAULT_AML_NCCL_SOCKET_IFNAME": "^docker0,lo"}),
    "profiling.constants": _section_constants("flops_profiler", "runtime.config", "FlopsProfilerConfig"),
    "nebula.constants": _section_constants("nebula", "nebula.config", "DeepSpeedNebulaConfig", extra={
        "NEBULA_EXPORT_ENVS": ["DLTS_JOB_ID", "DLTS_NUM_WORKER", "NEBULA_PERSISTENT_STORAGE_PATH",
                               "NEBULA_PERSISTENT_TIME_INTERVAL", "AML_RUN_ID", "AZUREML_RUN_TOKEN",
                               "AZUREML_WORKSPACE_SCOPE", "AZUREML_EXPERIMENT_SCOPE",
                               "AZUREML_RUN_HISTORY_SERVICE_ENDPOINT", "AZUREML_RUN_ID", "NEBULA_MEMORY_BUFFER_SIZE",
                               "AZUREML_PARAMETER_ITPJOB_NAME", "FC_TASKROLE_NAME", "FC_TASK_INDEX",
                               "MASTER_HOST", "LOCAL_HOST", "AZUREML_BLOB_ACCOUNT_NAME", "AZUREML_BLOB_ACCOUNT_KEY"],
        "DLTS_POD_ENV_PATH": "/dlts-runtime/env/pod.env"}),
    "autotuning.constants": _section_constants("autotuning", "autotuning.config", "DeepSpeedAutotuningConfig",
                                               extra={"AUTOTUNING_METRIC_LATENCY": "latency",
                                                      "AUTOTUNING_METRIC_THROUGHPUT": "throughput",
                                                      "AUTOTUNING_METRIC_FLOPS": "flops",
                                                      "AUTOTUNING_TUNER_GRIDSEARCH": "gridsearch",
                                                      "AUTOTUNING_TUNER_RANDOM": "random",
                                                      "AUTOTUNING_TUNER_MODELBASED": "model_based"}),
    "runtime.swap_tensor.constants": _section_constants("aio", "runtime.config", "AIOConfig"),
    "elasticity.constants": _section_constants("elasticity", "runtime.config", "ElasticityConfigModel", extra={
        "ENABLED": "enabled", "ENABLED_DEFAULT": False, "MAX_ACCEPTABLE_BATCH_SIZE": "max_train_batch_size",
        "MAX_ACCEPTABLE_BATCH_SIZE_DEFAULT": 2000, "MICRO_BATCHES": "micro_batch_sizes",
        "MICRO_BATCHES_DEFAULT": [2, 4, 6], "MIN_GPUS": "min_gpus", "MIN_GPUS_DEFAULT": 1, "MAX_GPUS": "max_gpus",
        "MAX_GPUS_DEFAULT": 10000, "NUM_GPUS_PER_NODE": "num_gpus_per_node", "NUM_GPUS_PER_NODE_DEFAULT": 1,
        "MODEL_PARALLEL_SIZE": "model_parallel_size", "MODEL_PARALLEL_SIZE_DEFAULT": 1, "MIN_TIME": "min_time",
        "MIN_TIME_DEFAULT": 0, "PREFER_LARGER_BATCH": "prefer_larger_batch", "PREFER_LARGER_BATCH_DEFAULT": True,
        "IGNORE_NON_ELASTIC_BATCH_INFO": "ignore_non_elastic_batch_info",
        "IGNORE_NON_ELASTIC_BATCH_INFO_DEFAULT": False, "VERSION": "version",
        "LATEST_ELASTICITY_VERSION": 0.2, "MINIMUM_DEEPSPEED_VERSION": "0.3.8",
        "DEEPSPEED_ELASTICITY_CONFIG": "DEEPSPEED_ELASTICITY_CONFIG"}),
}


_VIRTUAL = None


def _virtual_packages():
    """Proper prefixes of the served paths that are not served paths themselves."""
    global _VIRTUAL
    if _VIRTUAL is None:
        _VIRTUAL = set()
        for key in list(PATHS) + list(GENERATED):
            parts = key.split(".")
            for i in range(1, len(parts)):
                prefix = ".".join(parts[:i])
                if prefix not in PATHS and prefix not in GENERATED:
                    _VIRTUAL.add(prefix)
    return _VIRTUAL


def _has_children(rel):
    """A served path that other served paths lie below (the reference's `__init__.py` re-exports)."""
    return any(k.startswith(rel + ".") for k in list(PATHS) + list(GENERATED))


class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):

    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(_PKG + "."):
            return None
        rel = fullname[len(_PKG) + 1:]
        if rel in PATHS or rel in GENERATED:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=_has_children(rel))
        if rel in _virtual_packages():
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        return types.ModuleType(spec.name)

    def exec_module(self, module):
        rel = module.__name__[len(_PKG) + 1:]
        if rel in GENERATED:
            module.__doc__ = f"Reference constants module `deepspeed.{rel}`, derived from the config model."
            for k, v in GENERATED[rel]().items():
                setattr(module, k, v)
            return
        if rel not in PATHS:     # a directory of the reference's tree that only holds served paths
            module.__path__ = []
            module.__doc__ = f"Reference package `deepspeed.{rel}` (paths below it: `{_PKG}/_import_paths.py`)."
            return
        module.__doc__ = f"Reference import path `deepspeed.{rel}` (see `{_PKG}/_import_paths.py`)."
        if _has_children(rel):
            module.__path__ = []
        for real, names in PATHS[rel]:
            src = importlib.import_module(f"{_PKG}.{real}")
            if names == "*":
                for k, v in vars(src).items():
                    if not k.startswith("_"):
                        setattr(module, k, v)
            else:
                for exposed, actual in names.items():
                    if hasattr(src, actual):
                        setattr(module, exposed, getattr(src, actual))


def install():
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.append(_Finder())
