"""`offload_param` / `offload_optimizer` key constants at the reference's import path
(deepspeed/runtime/zero/offload_constants.py), generated from runtime/key_schema.py."""

from .. import key_schema as _ks
from .config import OFFLOAD_CPU_DEVICE, OFFLOAD_NVME_DEVICE  # noqa: F401

_params = [r for r in _ks.OFFLOAD if r[0].startswith("OFFLOAD_PARAM")]
_opt = [r for r in _ks.OFFLOAD if r[0].startswith("OFFLOAD_OPTIMIZER")]
globals().update(_ks.export(_params))
globals().update(_ks.export(_opt))
