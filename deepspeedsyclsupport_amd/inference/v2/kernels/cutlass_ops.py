"""Weight-only mixed GEMM and grouped MoE GEMM objects (reference `inference/v2/kernels/cutlass_ops/{mixed_gemm,
moe_gemm}`): the implementations live in `ops/cutlass_ops.py` on the gfx950 int8 / int4 streams and the grouped MFMA
GEMM."""
from ....ops.cutlass_ops import MixedGEMM, MixedMoEGEMM, MoEGEMM

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`

__all__ = ["MixedGEMM", "MoEGEMM", "MixedMoEGEMM"]
