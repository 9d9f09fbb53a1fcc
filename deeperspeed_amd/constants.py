"""Process-group defaults at the reference's import path (deepspeed/constants.py)."""

from datetime import timedelta

TORCH_DISTRIBUTED_DEFAULT_PORT = 29500
# torch.distributed's own default; the engine passes it to init_process_group
default_pg_timeout = timedelta(minutes=30)
