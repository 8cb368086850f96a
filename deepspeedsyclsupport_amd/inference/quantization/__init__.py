"""Weight-only group-wise int4 / int8 quantisation of an already built model (reference
`deepspeed/inference/quantization/`)."""
from .layers import QuantizedEmbedding, QuantizedLinear  # noqa: F401
from .quantization import _init_group_wise_weight_quantization  # noqa: F401
from .utils import DeQuantizer, Quantizer  # noqa: F401
