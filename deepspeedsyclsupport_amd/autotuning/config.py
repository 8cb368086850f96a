"""The `autotuning` section of the DeepSpeed config (reference `autotuning/config.py`, `autotuning/constants.py`)."""
from typing import Any, Dict, List, Optional

from ..runtime.config_utils import DeepSpeedConfigModel


class ModelInfoConfig(DeepSpeedConfigModel):
    profile: bool = False
    num_params: Optional[int] = None
    hidden_size: Optional[int] = None
    num_layers: Optional[int] = None


class DeepSpeedAutotuningConfig(DeepSpeedConfigModel):
    """Validated view of the section; `Autotuner` reads the same keys."""
    enabled: bool = False
    fast: bool = True
    results_dir: str = "autotuning_results"
    exps_dir: str = "autotuning_exps"
    overwrite: bool = True
    start_profile_step: int = 3
    end_profile_step: int = 5
    metric: str = "throughput"          # throughput | latency | flops
    metric_path: Optional[str] = None
    tuner_type: str = "gridsearch"      # gridsearch | random | model_based
    tuner_early_stopping: int = 5
    tuner_num_trials: int = 50
    arg_mappings: Optional[Dict[str, str]] = None
    mp_size: int = 1
    max_train_batch_size: Optional[int] = None
    min_train_batch_size: int = 1
    max_train_micro_batch_size_per_gpu: int = 1024
    min_train_micro_batch_size_per_gpu: int = 1
    num_tuning_micro_batch_sizes: int = 3
    zero_stages: List[int] = [0, 1, 2, 3]
    tuning_space: Optional[Dict[str, Any]] = None
    activation_mem_per_sample: Optional[int] = None
    model_info: Optional[ModelInfoConfig] = None
    model_info_path: Optional[str] = None

    def __init__(self, param_dict=None, **kw):
        if isinstance(param_dict, dict):   # the whole DeepSpeed config or the section itself
            kw = {**param_dict.get("autotuning", param_dict), **kw}
        super().__init__(**kw)


def get_default_model_info_config():
    return ModelInfoConfig().model_dump()


def get_model_info_config(param_dict):
    mi = (param_dict or {}).get("model_info")
    return ModelInfoConfig(**mi).model_dump() if mi else None
