"""ZeRO helpers (reference parity: deepspeed/runtime/zero/utils.py:1-46)."""

import torch
import torch.distributed as dist

from ...ops.adam.cpu_adam import DeepSpeedCPUAdam
from ...ops.adam.fused_adam import FusedAdam
from ...utils.logging import logger


def _initialize_parameter_parallel_groups(parameter_parallel_size=None):
    data_parallel_size = int(dist.get_world_size())
    parameter_parallel_size = parameter_parallel_size or data_parallel_size
    assert data_parallel_size % parameter_parallel_size == 0, \
        "world size should be divisible by parameter parallel size"
    rank = dist.get_rank()
    my_group = None
    for i in range(data_parallel_size // parameter_parallel_size):
        ranks = range(i * parameter_parallel_size, (i + 1) * parameter_parallel_size)
        group = dist.new_group(ranks)
        if rank in ranks:
            my_group = group
    return my_group


ZERO_SUPPORTED_OPTIMIZERS = [torch.optim.Adam, torch.optim.AdamW, FusedAdam, DeepSpeedCPUAdam]


def is_zero_supported_optimizer(optimizer):
    logger.info(f"Checking ZeRO support for optimizer={optimizer.__class__.__name__} type={type(optimizer)}")
    return type(optimizer) in ZERO_SUPPORTED_OPTIMIZERS
