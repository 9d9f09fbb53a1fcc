"""Config key constants at the reference's import path (deepspeed/runtime/constants.py).

Generated from runtime/key_schema.py, the table the config parser itself reads; pipeline
routes and precision/validation tables come from runtime/config.py."""

from . import key_schema as _ks
from .config import PRECISION_TYPES, SPARSE_MODE_DEFAULTS, ValidationMode  # noqa: F401

globals().update(_ks.export(_ks.TOP))

# pipeline engine routes (PipelineEngine.train_batch / eval_batch / inference_batch)
ROUTE_TRAIN, ROUTE_EVAL, ROUTE_PREDICT, ROUTE_ENCODE = "train", "eval", "predict", "encode"

SPARSE_DENSE_MODE, SPARSE_FIXED_MODE, SPARSE_VARIABLE_MODE = "dense", "fixed", "variable"
SPARSE_BIGBIRD_MODE, SPARSE_BSLONGFORMER_MODE = "bigbird", "bslongformer"
OPTIMIZER_TYPE_DEFAULT = SCHEDULER_TYPE_DEFAULT = None
FP32_ALLREDUCE_DEFAULT_BF16 = True  # bf16 runs reduce gradients in fp32 unless told otherwise
CHECKPOINT_TAG_VALIDATION_MODES = [m.value.capitalize() for m in ValidationMode]
