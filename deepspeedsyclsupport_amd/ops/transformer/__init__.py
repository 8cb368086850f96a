from . import functional  # noqa: F401
from .transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer, TransformerConfig  # noqa: F401
