from .quantizer import (ds_quantizer, quantize, dequantize, dequant_reduce, fake_quantize, QuantizedTensor)  # noqa
from .quantizer import (ds_quantize_fp32, ds_quantize_fp16, ds_sr_quantize_fp32, ds_sr_quantize_fp16,  # noqa
                        ds_quantize_asym_fp32, ds_quantize_asym_fp16, ds_sr_quantize_asym_fp32,
                        ds_sr_quantize_asym_fp16, dequantize_int4_to_half_experimental,
                        dequantize_int8_to_half_experimental, swizzle_quant, quantized_reduction)
