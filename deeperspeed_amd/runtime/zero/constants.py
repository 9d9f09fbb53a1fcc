"""`zero_optimization` key constants at the reference's import path
(deepspeed/runtime/zero/constants.py), generated from runtime/key_schema.py."""

from .. import key_schema as _ks
from .config import (MAX_STAGE_ZERO_OPTIMIZATION, ZERO_OPTIMIZATION_DISABLED, ZERO_OPTIMIZATION_GRADIENTS,  # noqa: F401
                     ZERO_OPTIMIZATION_OPTIMIZER_STATES, ZERO_OPTIMIZATION_WEIGHTS)

globals().update(_ks.export(_ks.ZERO))
ZERO_FORMAT = ZERO_OPTIMIZATION_FORMAT  # noqa: F821 (generated)
ZERO_OPTIMIZATION_STAGE_1, ZERO_OPTIMIZATION_STAGE_2, ZERO_OPTIMIZATION_STAGE_3 = 1, 2, 3
ZERO3_OPTIMIZATION_OVERLAP_COMM_DEFAULT = True
ZERO3_OPTIMIZATION_CONTIGUOUS_GRADIENTS_DEFAULT = True
ZERO_OPTIMIZATION_ALLGATHER_BUCKET_SIZE_DEPRECATED = "allgather_size"
ZERO_OPTIMIZATION_DEFAULT = _ks.defaults(_ks.ZERO)
