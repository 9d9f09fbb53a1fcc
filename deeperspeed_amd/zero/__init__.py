"""`deeperspeed_amd.zero` (reference: deepspeed/zero == deepspeed/runtime/zero/__init__.py)."""

from ..runtime.zero.partition_parameters import (GatheredParameters, Init, ZeroParamStatus, ZeroParamType,
                                                 register_external_parameter)
from ..runtime.zero.tiling import TiledLinear, TiledLinearReturnBias
from ..runtime.zero.linear import LinearFunctionForZeroStage3, LinearModuleForZeroStage3
from ..runtime.zero.contiguous_memory_allocator import ContiguousMemoryAllocator
from ..runtime.zero.compact_master import decode as compact_master_decode, encode as compact_master_encode
