"""Kernel objects of inference v2 (reference `inference/v2/kernels/`)."""
from .ds_kernel import DSKernelBase
from .core_ops import (BlasLibLinear, CUDABiasActivation, CUDAFPLN, CUDAFPPostLN, CUDAFPPreLN, CUDAGatedActivation,
                       CUDARMSNorm, CUDARMSPreNorm)
from .cutlass_ops import MixedGEMM, MixedMoEGEMM, MoEGEMM
from .ragged_ops import (AtomBuilder, BlockedFlashAttn, BlockedRotaryEmbeddings, BlockedTrainedRotaryEmbeddings,
                         LinearBlockedKVCopy, MoEGather, MoEScatter, RaggedEmbeddingKernel, RaggedLogitsGather,
                         RaggedTopKGating, get_kv_block_size, get_q_block_size)
