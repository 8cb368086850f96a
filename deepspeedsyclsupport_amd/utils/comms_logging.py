"""`deepspeed.utils.comms_logging` import path (reference `utils/comms_logging.py`): the comms logger lives in
`comm/comms_logging.py`."""
from ..comm.comms_logging import *  # noqa: F401,F403
