"""Training runtime (engine, ZeRO, pipeline, mixed precision, checkpoints)."""


class DeepSpeedOptimizer:
    """Marker base of every optimizer wrapper the engine builds (reference `runtime/__init__.py`)."""


class ZeROOptimizer(DeepSpeedOptimizer):
    """Marker base of the ZeRO optimizers (here: the one flat-group FlatZeroOptimizer for stages 0-3)."""
