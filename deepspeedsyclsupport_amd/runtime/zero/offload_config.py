"""offload_param / offload_optimizer sub-configs (reference `runtime/zero/offload_config.py:19-96`)."""
from enum import Enum
from typing import Optional

from pydantic import Field

from ..config_utils import DeepSpeedConfigModel


class OffloadDeviceEnum(str, Enum):
    none = "none"
    cpu = "cpu"
    nvme = "nvme"


class DeepSpeedZeroOffloadParamConfig(DeepSpeedConfigModel):
    device: OffloadDeviceEnum = "none"
    nvme_path: Optional[str] = None
    buffer_count: int = Field(5, ge=0)
    buffer_size: int = Field(int(1e8), ge=0)
    max_in_cpu: int = Field(int(1e9), ge=0)
    pin_memory: bool = False


class DeepSpeedZeroOffloadOptimizerConfig(DeepSpeedConfigModel):
    device: OffloadDeviceEnum = "none"
    nvme_path: Optional[str] = None
    buffer_count: int = Field(4, ge=0)
    pin_memory: bool = False
    pipeline_read: bool = False
    pipeline_write: bool = False
    fast_init: bool = False
    # ZeRO-Offload++ Twin-Flow: fraction of optimizer sub-groups stepped on the host (the rest on the GPU)
    ratio: float = Field(1.0, ge=0.0, le=1.0)
    # MI355X additions. With device "nvme": number of offloaded elements whose state stays in host DRAM (the rest is
    # streamed from NVMe), the optimizer-state analogue of offload_param.max_in_cpu.
    max_in_cpu: int = Field(0, ge=0)
    # let the next forward start while the host partition is still being stepped (modules wait for their own weights)
    overlap_forward: bool = False

    @property
    def pipeline(self):
        return self.pipeline_read or self.pipeline_write
