"""ZeRO stage 1 at the reference's import path (deepspeed/runtime/zero/stage1.py).

Stages 1 and 2 share one flat-arena implementation here (runtime/zero/stage_1_and_2.py)."""

from .stage_1_and_2 import FP16_DeepSpeedZeroOptimizer_Stage1  # noqa: F401
