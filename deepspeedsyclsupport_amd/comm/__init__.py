from .comm import *  # noqa: F401,F403
from .reduce_op import ReduceOp  # noqa: F401
