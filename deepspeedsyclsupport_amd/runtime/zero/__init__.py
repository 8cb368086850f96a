from .partition_parameters import Init, GatheredParameters, is_zero_param, shutdown_init_context  # noqa: F401
from .flat_optimizer import ZeroParamStatus, FlatZeroOptimizer  # noqa: F401
from .linear import LinearFunctionForZeroStage3, zero3_linear_wrap  # noqa: F401
from .config import DeepSpeedZeroConfig, ZeroStageEnum  # noqa: F401
from . import partition_parameters  # noqa: F401
