from .fused_lion import FusedLion  # noqa: F401
from .cpu_lion import DeepSpeedCPULion  # noqa: F401
