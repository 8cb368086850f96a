from torch.distributed import ReduceOp  # noqa: F401  (same enum RCCL/gloo consume)
