"""Process-group bring-up (reference parity: deepspeed/utils/distributed.py:12-142).

On MI355X the `"nccl"` backend of torch.distributed is RCCL (xGMI intra-node).  When no
GPU is visible (CPU CI) the requested backend is transparently mapped to `gloo` so the
same multi-process code paths run in tests.
"""

import os
from datetime import timedelta

import torch

from .logging import logger

default_pg_timeout = timedelta(minutes=int(os.environ.get("DSA_PG_TIMEOUT_MIN", "30")))


def _resolve_backend(backend):
    if backend in (None, "nccl", "rccl") and not torch.cuda.is_available():
        return "gloo"
    if backend == "rccl":
        return "nccl"
    return backend or "nccl"


def init_distributed(dist_backend="nccl", auto_mpi_discovery=True, distributed_port=29500, verbose=True,
                     timeout=default_pg_timeout, init_method=None):
    """Initialise torch.distributed from env vars (RANK/WORLD_SIZE/MASTER_*), falling back
    to MPI discovery (OMPI_* env / mpi4py) or Azure ML env when required vars are missing."""
    import torch.distributed as dist
    required_env = ["RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_RANK"]
    if auto_mpi_discovery and not all(v in os.environ for v in required_env):
        if in_aml() and not in_dlts():
            patch_aml_env_for_torch_nccl_backend(master_port=distributed_port, verbose=verbose)
        else:
            mpi_discovery(distributed_port=distributed_port, verbose=verbose)
    for v, d in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"), ("MASTER_ADDR", "127.0.0.1"),
                 ("MASTER_PORT", str(distributed_port))):
        os.environ.setdefault(v, d)
    # failed / timed-out RCCL collectives abort the process (the launcher then tears the job
    # down) instead of hanging every rank
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]) % max(1, torch.cuda.device_count()))
    if not dist.is_initialized():
        backend = _resolve_backend(dist_backend)
        if verbose:
            logger.info("Initializing torch distributed with backend: {} (rank {}/{})".format(
                backend, os.environ["RANK"], os.environ["WORLD_SIZE"]))
        kwargs = dict(backend=backend, timeout=timeout, init_method=init_method,
                      rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
        if backend == "nccl" and torch.cuda.is_available():
            kwargs["device_id"] = torch.device("cuda", torch.cuda.current_device())
            # RCCL on high-priority HIP streams: ZeRO's all-gathers / reduce-scatters are
            # scheduled ahead of the compute kernels they overlap with, so a prefetch does not
            # queue behind a long GEMM
            try:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kwargs["pg_options"] = opts
            except (AttributeError, RuntimeError):
                pass
        try:
            dist.init_process_group(**kwargs)
        except TypeError:
            kwargs.pop("device_id", None)
            kwargs.pop("pg_options", None)
            dist.init_process_group(**kwargs)


def mpi_discovery(distributed_port=29500, verbose=True):
    """Discover rank/world/master from an MPI launch (mpi4py if present, else OMPI_* env)."""
    rank = world_size = local_rank = None
    master_addr = None
    try:
        from mpi4py import MPI  # optional
        comm = MPI.COMM_WORLD
        rank = comm.Get_rank()
        world_size = comm.Get_size()
        import subprocess
        master_addr = None
        if rank == 0:
            master_addr = subprocess.check_output("hostname -I", shell=True).decode().split()[0]
        master_addr = comm.bcast(master_addr, root=0)
        import socket
        proc_name = socket.gethostname()
        all_procs = comm.allgather(proc_name)
        local_rank = sum([i == proc_name for i in all_procs[:rank]])
    except ImportError:
        if "OMPI_COMM_WORLD_RANK" in os.environ:
            rank = int(os.environ["OMPI_COMM_WORLD_RANK"])
            world_size = int(os.environ["OMPI_COMM_WORLD_SIZE"])
            local_rank = int(os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", "0"))
        elif "SLURM_PROCID" in os.environ:
            rank = int(os.environ["SLURM_PROCID"])
            world_size = int(os.environ["SLURM_NTASKS"])
            local_rank = int(os.environ.get("SLURM_LOCALID", "0"))
        else:
            return
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world_size)
    os.environ["LOCAL_RANK"] = str(local_rank)
    if master_addr:
        os.environ["MASTER_ADDR"] = master_addr
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(distributed_port)
    if verbose:
        logger.info("Discovered MPI settings of world_rank={}, local_rank={}, world_size={}, master_addr={}, "
                    "master_port={}".format(rank, local_rank, world_size, os.environ["MASTER_ADDR"],
                                            os.environ["MASTER_PORT"]))


def in_aml():
    return "AZUREML_EXPERIMENT_ID" in os.environ


def in_dlts():
    return "DLTS_JOB_ID" in os.environ


def patch_aml_env_for_torch_nccl_backend(master_port=6105, verbose=True):
    os.environ["RANK"] = os.environ["OMPI_COMM_WORLD_RANK"]
    os.environ["WORLD_SIZE"] = os.environ["OMPI_COMM_WORLD_SIZE"]
    single_node = int(os.environ["OMPI_COMM_WORLD_LOCAL_SIZE"]) == int(os.environ["WORLD_SIZE"])
    if not single_node:
        master_node_params = os.environ["AZ_BATCH_MASTER_NODE"].split(":")
        os.environ["MASTER_ADDR"] = master_node_params[0]
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(master_port)
    else:
        os.environ["MASTER_ADDR"] = os.environ["AZ_BATCHAI_MPI_MASTER_NODE"]
        os.environ["MASTER_PORT"] = "54965"
    os.environ["LOCAL_RANK"] = os.environ["OMPI_COMM_WORLD_LOCAL_RANK"]
    if verbose:
        logger.info("AML env: RANK={} LOCAL_RANK={} WORLD_SIZE={} MASTER_ADDR={} MASTER_PORT={}".format(
            os.environ["RANK"], os.environ["LOCAL_RANK"], os.environ["WORLD_SIZE"], os.environ["MASTER_ADDR"],
            os.environ["MASTER_PORT"]))
