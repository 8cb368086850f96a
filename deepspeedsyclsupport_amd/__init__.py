"""deepspeedsyclsupport_amd — an MI355X-native (gfx950 / ROCm / RCCL-over-xGMI) ZeRO training & inference framework
with the capabilities and user API of DeepSpeed (`deepspeed.initialize`, `engine.backward/step`, `zero.Init`,
`init_inference`, ...). See SURVEY.md for the component map and README.md for the design."""
# API level of the reference release this framework tracks (scripts and elasticity checks compare against it);
# the MI355X implementation has its own release counter.
__version__ = "0.12.7"
__mi355x_version__ = "0.1.0"
version = __version__
__version_major__, __version_minor__, __version_patch__ = 0, 12, 7
__git_hash__ = None
__git_branch__ = None

import torch  # noqa: E402

from . import _import_paths  # noqa: E402

_import_paths.install()  # reference module paths that are folded into other files here
from . import comm  # noqa: E402,F401
from . import comm as dist  # noqa: E402,F401
from .accelerator import get_accelerator  # noqa: E402,F401
from .comm import init_distributed  # noqa: E402,F401
from .runtime import zero  # noqa: E402,F401
from .runtime.config import DeepSpeedConfig, DeepSpeedConfigError  # noqa: E402,F401
from .runtime.engine import DeepSpeedEngine  # noqa: E402,F401
from .runtime.lr_schedules import add_tuning_arguments  # noqa: E402,F401
from .utils.logging import log_dist, logger  # noqa: E402,F401

# reference type aliases for the `optimizer=` / `lr_scheduler=` callables of `initialize`
from typing import Callable, Iterable, Union  # noqa: E402

DeepSpeedOptimizerCallable = Callable[[Union[Iterable[torch.nn.Parameter], dict]], torch.optim.Optimizer]
DeepSpeedSchedulerCallable = Callable[[torch.optim.Optimizer], object]


# the rest of the reference's top-level names, imported on first use (keeps `import` light and cycle-free)
_LAZY = {
    "ops": (".ops", None),
    "module_inject": (".module_inject", None),
    "DeepSpeedHybridEngine": (".runtime.hybrid_engine", "DeepSpeedHybridEngine"),
    "PipelineEngine": (".runtime.pipe.engine", "PipelineEngine"),
    "PipelineModule": (".runtime.pipe.module", "PipelineModule"),
    "InferenceEngine": (".inference.engine", "InferenceEngine"),
    "DeepSpeedInferenceConfig": (".inference.config", "DeepSpeedInferenceConfig"),
    "checkpointing": (".runtime.activation_checkpointing", "checkpointing"),
    "DeepSpeedTransformerLayer": (".ops.transformer", "DeepSpeedTransformerLayer"),
    "DeepSpeedTransformerConfig": (".ops.transformer", "DeepSpeedTransformerConfig"),
    "replace_transformer_layer": (".module_inject.replace_module", "replace_transformer_layer"),
    "revert_transformer_layer": (".module_inject.replace_module", "revert_transformer_layer"),
    "OnDevice": (".utils.init_on_device", "OnDevice"),
    "DeepSpeedOptimizer": (".runtime", "DeepSpeedOptimizer"),
    "ZeROOptimizer": (".runtime", "ZeROOptimizer"),
    "ADAM_OPTIMIZER": (".runtime.config", "ADAM_OPTIMIZER"),
    "LAMB_OPTIMIZER": (".runtime.config", "LAMB_OPTIMIZER"),
}
git_hash, git_branch = __git_hash__, __git_branch__


def __getattr__(name):
    if name not in _LAZY:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    import importlib
    mod, attr = _LAZY[name]
    m = importlib.import_module(mod, __name__)
    val = m if attr is None else getattr(m, attr)
    globals()[name] = val
    return val


def _parse_version(s):
    return tuple(int(x) for x in s.split(".")[:3])


def initialize(args=None, model=None, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
               mpu=None, dist_init_required=None, collate_fn=None, config=None, config_params=None):
    """Build the training engine (reference `deepspeed/__init__.py:64-202`).

    Returns (engine, optimizer, training_dataloader, lr_scheduler)."""
    log_dist(f"DeepSpeed-AMD info: version={__version__}", ranks=[0])
    assert model is not None, "deepspeed.initialize requires a model"
    zero.partition_parameters.shutdown_init_context()
    if config is None and config_params is not None:
        config = config_params
    if config is None and args is not None:
        config = getattr(args, "deepspeed_config", None)
    assert config is not None, "DeepSpeed requires --deepspeed_config or config=..."
    if args is not None and getattr(args, "deepspeed_mpi", False):
        comm.mpi_discovery()
    if dist_init_required is not False:
        init_distributed(dist_init_required=dist_init_required)
    try:
        from .runtime.pipe.module import PipelineModule
        pipe = isinstance(model, PipelineModule)
    except ImportError:
        pipe = False
    cfg = config if isinstance(config, DeepSpeedConfig) else \
        DeepSpeedConfig(config, model.mpu() if pipe else mpu)
    wq = cfg.param_dict.get("weight_quantization") or {}
    if wq.get("quantized_initialization"):
        # reference `runtime/zero/partition_parameters.py:317`: every linear / embedding weight is held as group-wise
        # int4 / int8 codes; here the pass runs over the built model before the engine takes it
        from .inference.quantization import _init_group_wise_weight_quantization
        _init_group_wise_weight_quantization(
            model, {"weight_quantization": {"quantized_initialization": wq["quantized_initialization"]}})
    if pipe:
        from .runtime.pipe.engine import PipelineEngine
        engine = PipelineEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                training_data=training_data, lr_scheduler=lr_scheduler, mpu=model.mpu(),
                                dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                                config_class=cfg)
    elif cfg.hybrid_engine.enabled:
        from .runtime.hybrid_engine import DeepSpeedHybridEngine
        engine = DeepSpeedHybridEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                       training_data=training_data, lr_scheduler=lr_scheduler, mpu=mpu,
                                       dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                                       config_class=cfg)
    else:
        engine = DeepSpeedEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                 training_data=training_data, lr_scheduler=lr_scheduler, mpu=mpu,
                                 dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                                 config_class=cfg)
    zero.partition_parameters.restore_init_context()
    return engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler


def _add_core_arguments(parser):
    group = parser.add_argument_group("DeepSpeed", "DeepSpeed configurations")
    group.add_argument("--deepspeed", default=False, action="store_true", help="Enable DeepSpeed")
    group.add_argument("--deepspeed_config", default=None, type=str, help="DeepSpeed json configuration file.")
    group.add_argument("--deepscale", default=False, action="store_true", help=argparse_suppress())
    group.add_argument("--deepscale_config", default=None, type=str, help=argparse_suppress())
    group.add_argument("--deepspeed_mpi", default=False, action="store_true",
                       help="Run via MPI, this will attempt to discover the necessary variables to initialize "
                       "torch distributed from the MPI environment")
    return parser


def argparse_suppress():
    import argparse
    return argparse.SUPPRESS


def add_config_arguments(parser):
    return _add_core_arguments(parser)


def default_inference_config():
    from .inference.config import DeepSpeedInferenceConfig
    return DeepSpeedInferenceConfig().model_dump()


def init_inference(model, config=None, **kwargs):
    """Inference engine with kernel injection / AutoTP (reference `deepspeed/__init__.py:269-344`)."""
    from .inference.config import DeepSpeedInferenceConfig
    from .inference.engine import InferenceEngine
    if config is None:
        config = {}
    if isinstance(config, str):
        import json
        with open(config) as f:
            config = json.load(f)
    if isinstance(config, dict):
        overlap = set(config) & set(kwargs)
        for k in overlap:
            if config[k] != kwargs[k]:
                raise ValueError(f"Conflicting argument '{k}' in 'config':{config[k]} and kwargs:{kwargs[k]}")
        config = {**config, **kwargs}
        ds_inference_config = DeepSpeedInferenceConfig(**config)
    else:
        ds_inference_config = config
    return InferenceEngine(model, config=ds_inference_config)
