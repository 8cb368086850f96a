from .logging import logger, log_dist  # noqa: F401
from .nvtx import instrument_w_nvtx  # noqa: F401
