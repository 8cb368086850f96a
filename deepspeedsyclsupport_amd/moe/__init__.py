from .layer import MoE  # noqa: F401
