"""`deepspeed.utils.groups` import path (reference `utils/groups.py`): the process-group topology lives in
`parallel/groups.py`; this module re-exports it so scripts written against the reference path work unchanged."""
from ..parallel.groups import *  # noqa: F401,F403
from ..parallel import groups as _impl

mpu = None


def __getattr__(name):
    return getattr(_impl, name)
