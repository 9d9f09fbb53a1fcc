"""Reference import path (deepspeed/runtime/fp16/fused_optimizer.py: `FP16_Optimizer`).
The flat-master fp16/bf16 wrapper is the stage-0 flat-arena optimizer."""

from ..zero.stage_1_and_2 import FP16_Optimizer  # noqa: F401
