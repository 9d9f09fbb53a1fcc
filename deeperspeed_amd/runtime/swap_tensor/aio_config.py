"""`aio` section parsing at the reference's import path (deepspeed/runtime/swap_tensor/aio_config.py)."""

from ..config import get_aio_config  # noqa: F401
