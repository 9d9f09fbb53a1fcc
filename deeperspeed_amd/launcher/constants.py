"""Launcher constants (reference parity: deepspeed/launcher/constants.py)."""

PDSH_LAUNCHER = "pdsh"
PDSH_MAX_FAN_OUT = 1024
OPENMPI_LAUNCHER = "openmpi"
SLURM_LAUNCHER = "slurm"
MVAPICH_LAUNCHER = "mvapich"
MOSAICML_LAUNCHER = "mosaicml"
MVAPICH_TMP_HOSTFILE = "/tmp/deeperspeed_amd_mvapich_hostfile"
TORCH_DISTRIBUTED_DEFAULT_PORT = 29500
DEFAULT_HOSTFILE = "/job/hostfile"
# environment propagated to every node (reference runner.py:27-30 + the ROCm stack)
EXPORT_ENVS = ["NCCL", "RCCL", "HSA", "HIP", "ROCM", "GPU_MAX_HW_QUEUES", "PYTHON", "MV2", "UCX", "OMP", "TORCH",
               "PYTORCH", "DSA_"]
DEEPSPEED_ENVIRONMENT_NAME = ".deepspeed_env"
