"""Model compression (QAT, pruning, layer reduction) — reference `deepspeed/compression/`."""
from .basic_layer import (BNLayer_Compress, ColumnParallelLinear_Compress, Conv2dLayer_Compress, Embedding_Compress,
                          LinearLayer_Compress, QuantAct, RowParallelLinear_Compress, fake_quant)
from .compress import init_compression, redundancy_clean, student_initialization
from .config import get_compression_config
from .helper import convert_conv1d_to_linear, fix_compression, module_replacement, recursive_getattr, \
    recursive_setattr
from .scheduler import compression_scheduler
from .utils import AsymQuantizer, BinaryQuantizer, SymQuantizer, TernaryQuantizer, TopKBinarizer
