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
    "runtime.zero.stage3": [("runtime.zero.flat_optimizer", {"DeepSpeedZeroOptimizer_Stage3": "DeepSpeedZeroOptimizer_Stage3"})],
    "runtime.zero.stage_1_and_2": [("runtime.zero.flat_optimizer", {"DeepSpeedZeroOptimizer": "DeepSpeedZeroOptimizer"})],
    "runtime.zero.partitioned_param_coordinator": [("runtime.zero.coordinator",
                                                    {"PartitionedParameterCoordinator": "ParamCoordinator"})],
    "runtime.zero.parameter_offload": [("runtime.zero.coordinator", {"DeepSpeedZeRoOffload": "ParamCoordinator"})],
    "runtime.zero.mics": [("runtime.zero", {"MiCS_Init": "MiCS_Init", "MiCS_Optimizer": "MiCS_Optimizer"})],
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
}


class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):

    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(_PKG + "."):
            return None
        if fullname[len(_PKG) + 1:] in PATHS:
            return importlib.machinery.ModuleSpec(fullname, self)
        return None

    def create_module(self, spec):
        return types.ModuleType(spec.name)

    def exec_module(self, module):
        rel = module.__name__[len(_PKG) + 1:]
        module.__doc__ = f"Reference import path `deepspeed.{rel}` (see `{_PKG}/_import_paths.py`)."
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
