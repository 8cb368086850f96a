"""Model compression (QAT, pruning, layer reduction) — reference `deepspeed/compression/`."""
from .basic_layer import Embedding_Compress, LinearLayer_Compress, QuantAct, fake_quant
from .compress import compression_scheduler, init_compression, redundancy_clean, student_initialization
