from .logging import logger, log_dist  # noqa: F401
from .nvtx import instrument_w_nvtx  # noqa: F401
from .tensor_fragment import (safe_get_full_fp32_param, safe_get_full_grad, safe_get_full_optimizer_state,  # noqa
                              safe_get_local_fp32_param, safe_get_local_grad, safe_get_local_optimizer_state,
                              safe_set_full_fp32_param, safe_set_full_optimizer_state)
