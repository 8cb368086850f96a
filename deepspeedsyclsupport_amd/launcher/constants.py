"""Launcher constants (reference `launcher/constants.py`)."""
PDSH_LAUNCHER = "pdsh"
PDSH_MAX_FAN_OUT = 1024
OPENMPI_LAUNCHER = "openmpi"
MPICH_LAUNCHER = "mpich"
IMPI_LAUNCHER = "impi"
SLURM_LAUNCHER = "slurm"
MVAPICH_LAUNCHER = "mvapich"
MVAPICH_TMP_HOSTFILE = "/tmp/deepspeed_mvapich_hostfile"
ELASTIC_TRAINING_ID_DEFAULT = "123456789"
DEFAULT_HOSTFILE = "/job/hostfile"
TORCH_DISTRIBUTED_DEFAULT_PORT = 29500
# environment prefixes forwarded to remote nodes (ROCm / RCCL / HIP instead of CUDA / NCCL-only)
EXPORT_ENVS = ["MLFLOW", "PYTHON", "MV2", "UCX", "NCCL", "RCCL", "HIP", "HSA", "ROCR", "ROCM", "MIOPEN", "OMP",
               "DS_", "TORCH"]
