from . import checkpointing  # noqa: F401
from .checkpointing import checkpoint, configure, is_configured  # noqa: F401
