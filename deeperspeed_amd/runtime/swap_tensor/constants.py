"""`aio` key constants at the reference's import path (deepspeed/runtime/swap_tensor/constants.py)."""

from .. import key_schema as _ks

globals().update(_ks.export(_ks.AIO))
