from .checkpoint_engine import CheckpointEngine, TorchCheckpointEngine, AsyncCheckpointEngine  # noqa: F401
