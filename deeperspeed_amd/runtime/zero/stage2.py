"""ZeRO stage 2 at the reference's import path (deepspeed/runtime/zero/stage2.py).

Stages 1 and 2 share one flat-arena implementation here (runtime/zero/stage_1_and_2.py)."""

from .stage_1_and_2 import DeepSpeedZeroOptimizer, FP16_DeepSpeedZeroOptimizer  # noqa: F401
