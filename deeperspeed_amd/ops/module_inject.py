"""Legacy import path of the layer-injection helpers (reference deepspeed/ops/module_inject.py)."""

from ..module_inject.replace_module import (module_inject, replace_module, replace_transformer_layer,  # noqa: F401
                                            revert_transformer_layer)
