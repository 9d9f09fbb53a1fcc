"""`deeperspeed_amd.checkpointing` (reference: `deepspeed.checkpointing` alias of
deepspeed/runtime/activation_checkpointing/checkpointing.py)."""

from .runtime.activation_checkpointing.checkpointing import *  # noqa: F401,F403
from .runtime.activation_checkpointing.checkpointing import (checkpoint, configure, get_cuda_rng_tracker,
                                                             is_configured, model_parallel_cuda_manual_seed,
                                                             partition_activations_in_checkpoint, reset)
