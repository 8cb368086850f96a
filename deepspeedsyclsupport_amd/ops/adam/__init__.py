from .fused_adam import FusedAdam, adam_flat_update  # noqa: F401
from .cpu_adam import DeepSpeedCPUAdam  # noqa: F401
