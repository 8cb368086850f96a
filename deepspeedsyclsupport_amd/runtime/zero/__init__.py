from .partition_parameters import (Init, GatheredParameters, is_zero_param, shutdown_init_context,  # noqa: F401
                                   restore_init_context, register_external_parameter,
                                   unregister_external_parameter)
from .flat_optimizer import ZeroParamStatus, FlatZeroOptimizer  # noqa: F401
from .linear import LinearFunctionForZeroStage3, zero3_linear_wrap  # noqa: F401
from .config import DeepSpeedZeroConfig, ZeroStageEnum  # noqa: F401
from . import partition_parameters  # noqa: F401
from .tiling import TiledLinear, TiledLinearReturnBias  # noqa: F401
from .zeropp import quantized_all_gather, quantized_reduce_scatter  # noqa: F401

# MiCS (reference `runtime/zero/mics.py`): the flat-group optimizer implements MiCS when `mics_shard_size` is set;
# `MiCS_Init` partitions exactly like `Init` (the shard group is chosen by the optimizer at engine init).
MiCS_Init = Init
MiCS_Optimizer = FlatZeroOptimizer
