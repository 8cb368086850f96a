from .quantizer import (ds_quantizer, quantize, dequantize, dequant_reduce, fake_quantize, QuantizedTensor)  # noqa
