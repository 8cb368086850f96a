"""The `nebula` section of the DeepSpeed config (reference `nebula/config.py`, `nebula/constants.py`)."""
from typing import Optional

from ..runtime.config_utils import DeepSpeedConfigModel


class DeepSpeedNebulaConfig(DeepSpeedConfigModel):
    enabled: bool = False
    load_path: Optional[str] = None
    enable_nebula_load: bool = True
    persistent_storage_path: Optional[str] = None
    persistent_time_interval: int = 100
    num_of_version_in_retention: int = 2

    def __init__(self, param_dict=None, **kw):
        if isinstance(param_dict, dict):
            kw = {**param_dict.get("nebula", param_dict), **kw}
        super().__init__(**kw)
