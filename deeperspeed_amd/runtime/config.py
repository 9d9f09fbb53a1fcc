"""DeepSpeed JSON configuration.

Reference parity: deepspeed/runtime/config.py:536-812 and runtime/constants.py (full key
surface of SURVEY §2.6, including the DeeperSpeed deltas: `fp16.type = "bfloat16"` with
loss scale forced to 1.0, and `fp32_allreduce` defaulting to true for bf16).

Structure here: a declarative table of top-level scalar keys plus small section parsers;
`DeepSpeedConfig` resolves the batch triple (train = micro * gas * dp_world) and
elasticity overrides, then validates.
"""

import copy
import json
from enum import Enum

import torch

from ..elasticity import compute_elastic_config, elasticity_enabled, ensure_immutable_elastic_config
from ..elasticity.config import ElasticityConfigError
from ..elasticity.constants import (ELASTICITY, IGNORE_NON_ELASTIC_BATCH_INFO, IGNORE_NON_ELASTIC_BATCH_INFO_DEFAULT)
from ..utils.logging import logger
from ..version import __version__
from .activation_checkpointing.config import DeepSpeedActivationCheckpointingConfig
from .config_utils import ScientificNotationEncoder, dict_raise_error_on_duplicate_keys
from .zero.config import DeepSpeedZeroConfig, MAX_STAGE_ZERO_OPTIMIZATION

# ---------------------------------------------------------------------------------- keys
TRAIN_BATCH_SIZE = "train_batch_size"
TRAIN_MICRO_BATCH_SIZE_PER_GPU = "train_micro_batch_size_per_gpu"
GRADIENT_ACCUMULATION_STEPS = "gradient_accumulation_steps"

ADAM_OPTIMIZER = "adam"
ADAMW_OPTIMIZER = "adamw"
LAMB_OPTIMIZER = "lamb"
ONEBIT_ADAM_OPTIMIZER = "onebitadam"
ONEBIT_LAMB_OPTIMIZER = "onebitlamb"
DEEPSPEED_OPTIMIZERS = [ADAM_OPTIMIZER, ADAMW_OPTIMIZER, LAMB_OPTIMIZER, ONEBIT_ADAM_OPTIMIZER,
                        ONEBIT_LAMB_OPTIMIZER]
TORCH_ADAM_PARAM = "torch_adam"
ADAM_W_MODE = "adam_w_mode"
ADAM_W_MODE_DEFAULT = True
MAX_GRAD_NORM = "max_grad_norm"

PRECISION_TYPES = {
    "fp32": torch.float32, "float32": torch.float32, "float": torch.float32,
    "fp16": torch.half, "float16": torch.half, "half": torch.half,
    "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
}

TENSOR_CORE_ALIGN_SIZE = 8

# top-level scalar keys -> (attribute, default)
_TOP_LEVEL = {
    "steps_per_print": ("steps_per_print", 10),
    "dump_state": ("dump_state", False),
    "disable_allgather": ("disable_allgather", False),
    "prescale_gradients": ("prescale_gradients", False),
    "gradient_predivide_factor": ("gradient_predivide_factor", 1.0),
    "sparse_gradients": ("sparse_gradients_enabled", False),
    "gradient_clipping": ("gradient_clipping", 0.0),
    "zero_allow_untested_optimizer": ("zero_allow_untested_optimizer", False),
    "wall_clock_breakdown": ("wall_clock_breakdown", False),
    "memory_breakdown": ("memory_breakdown", False),
}

# sparse attention (constants.py:24-55)
SPARSE_ATTENTION = "sparse_attention"
SPARSE_MODE_DEFAULTS = {
    "dense": dict(block=16),
    "fixed": dict(block=16, different_layout_per_head=False, num_local_blocks=4, num_global_blocks=1,
                  attention="bidirectional", horizontal_global_attention=False, num_different_global_patterns=1),
    "variable": dict(block=16, different_layout_per_head=False, num_random_blocks=0, local_window_blocks=[4],
                     global_block_indices=[0], global_block_end_indices=None, attention="bidirectional",
                     horizontal_global_attention=False),
    "bigbird": dict(block=16, different_layout_per_head=False, num_random_blocks=1, num_sliding_window_blocks=3,
                    num_global_blocks=1),
    "bslongformer": dict(block=16, different_layout_per_head=False, num_sliding_window_blocks=3,
                         global_block_indices=[0], global_block_end_indices=None),
    "local_sliding_window": dict(block=16, num_sliding_window_blocks=3, attention="unidirectional"),
}

PIPELINE_DEFAULTS = {"stages": "auto", "partition": "best", "seed_layers": False, "activation_checkpoint_interval": 0}


class ValidationMode(Enum):
    WARN = "WARN"
    IGNORE = "IGNORE"
    FAIL = "FAIL"


class DeepSpeedConfigError(Exception):
    pass


# ---------------------------------------------------------------------------------- sections
def _fp16_section(param_dict):
    d = param_dict.get("fp16", {}) or {}
    enabled = bool(d.get("enabled", False))
    ftype = str(d.get("type", "fp16")).lower()
    if ftype not in PRECISION_TYPES:
        raise DeepSpeedConfigError(f"unknown fp16.type {ftype}")
    precision = PRECISION_TYPES[ftype]
    # bf16 needs no loss scaling: DeeperSpeed forces the static scale to 1.0 (config.py:106-108)
    if enabled and precision == torch.bfloat16:
        loss_scale = 1.0
    else:
        loss_scale = d.get("loss_scale", 0) if enabled else 0
    init_power = d.get("initial_scale_power", 32)
    dyn_args = None
    if enabled:
        dyn_args = {
            "init_scale": 2 ** init_power,
            "scale_window": d.get("loss_scale_window", 1000),
            "delayed_shift": d.get("hysteresis", 2),
            "min_scale": d.get("min_loss_scale", 1),
        }
    return enabled, ftype, precision, loss_scale, 2 ** init_power, dyn_args


def _sparse_attention_section(param_dict):
    if SPARSE_ATTENTION not in param_dict:
        return None
    sd = param_dict[SPARSE_ATTENTION]
    mode = sd.get("mode", "fixed")
    if mode not in SPARSE_MODE_DEFAULTS:
        raise NotImplementedError(f"Given sparsity mode, {mode}, has not been implemented yet!")
    out = {"mode": mode}
    for k, v in SPARSE_MODE_DEFAULTS[mode].items():
        out[k] = sd.get(k, copy.deepcopy(v))
    return out


def _pipeline_section(param_dict):
    out = dict(PIPELINE_DEFAULTS)
    out.update(param_dict.get("pipeline", {}) or {})
    return out


class DeepSpeedFlopsProfilerConfig:
    """`flops_profiler` section (reference: profiling/config.py, profiling/constants.py:24-39)."""

    def __init__(self, param_dict):
        d = param_dict.get("flops_profiler", {}) or {}
        self.enabled = d.get("enabled", False)
        self.profile_step = d.get("profile_step", 1)
        self.module_depth = d.get("module_depth", -1)
        self.top_modules = d.get("top_modules", 3)
        self.detailed = d.get("detailed", True)


def get_aio_config(param_dict):
    """`aio` section (reference: swap_tensor/aio_config.py, constants.py:17-27)."""
    d = param_dict.get("aio", {}) or {}
    return {
        "block_size": d.get("block_size", 1048576),
        "queue_depth": d.get("queue_depth", 8),
        "thread_count": d.get("thread_count", 1),
        "single_submit": d.get("single_submit", False),
        "overlap_events": d.get("overlap_events", True),
    }


# ---------------------------------------------------------------------------------- main
class DeepSpeedConfig:
    def __init__(self, json_file=None, mpu=None, param_dict=None):
        if param_dict is None:
            if isinstance(json_file, dict):
                param_dict = json_file
            else:
                with open(json_file, "r") as f:
                    param_dict = json.load(f, object_pairs_hook=dict_raise_error_on_duplicate_keys)
        self._param_dict = param_dict
        try:
            import torch.distributed as dist
            self.global_rank = dist.get_rank()
            self.world_size = mpu.get_data_parallel_world_size() if mpu is not None else dist.get_world_size()
        except Exception:
            self.global_rank, self.world_size = 0, 1

        self.elasticity_enabled = elasticity_enabled(self._param_dict)
        if self.elasticity_enabled:
            self._apply_elasticity()
        self._initialize_params(self._param_dict)
        self._configure_train_batch_size()
        self._do_sanity_check()

    # ---------------------------------------------------------------- elasticity
    def _apply_elasticity(self):
        logger.info("DeepSpeed elasticity support enabled")
        final_bs, valid_gpus, micro = compute_elastic_config(ds_config=self._param_dict,
                                                             target_deepspeed_version=__version__,
                                                             world_size=self.world_size)
        ed = self._param_dict[ELASTICITY]
        ensure_immutable_elastic_config(runtime_elastic_config_dict=ed)
        if not ed.get(IGNORE_NON_ELASTIC_BATCH_INFO, IGNORE_NON_ELASTIC_BATCH_INFO_DEFAULT):
            batch_keys = [TRAIN_BATCH_SIZE, TRAIN_MICRO_BATCH_SIZE_PER_GPU, GRADIENT_ACCUMULATION_STEPS]
            if any(k in self._param_dict for k in batch_keys):
                raise ElasticityConfigError(
                    "One or more batch related parameters were found in your ds_config "
                    f"({TRAIN_BATCH_SIZE}, {TRAIN_MICRO_BATCH_SIZE_PER_GPU}, and/or {GRADIENT_ACCUMULATION_STEPS}). "
                    "These parameters *will not be used* since elastic training is enabled. Set "
                    f"'{IGNORE_NON_ELASTIC_BATCH_INFO}': true to silently ignore them.")
        gas = final_bs // (micro * self.world_size)
        logger.info(f"[Elasticity] valid GPU counts: {valid_gpus}")
        self._param_dict[TRAIN_BATCH_SIZE] = final_bs
        self._param_dict[TRAIN_MICRO_BATCH_SIZE_PER_GPU] = micro
        self._param_dict[GRADIENT_ACCUMULATION_STEPS] = gas

    # ---------------------------------------------------------------- parse
    def _initialize_params(self, pd):
        self.train_batch_size = pd.get(TRAIN_BATCH_SIZE)
        self.train_micro_batch_size_per_gpu = pd.get(TRAIN_MICRO_BATCH_SIZE_PER_GPU)
        self.gradient_accumulation_steps = pd.get(GRADIENT_ACCUMULATION_STEPS)
        for key, (attr, default) in _TOP_LEVEL.items():
            setattr(self, attr, pd.get(key, default))

        (self.fp16_enabled, self.fp16_type, self.precision, self.loss_scale, self.initial_dynamic_scale,
         self.dynamic_loss_scale_args) = _fp16_section(pd)
        self.bfloat16_enabled = self.fp16_enabled and self.precision == torch.bfloat16
        # DeeperSpeed: fp32 communication defaults ON for bf16 (config.py:180-184)
        default_fp32_ar = self.fp16_enabled and self.precision == torch.bfloat16
        self.allreduce_always_fp32 = pd.get("fp32_allreduce", default_fp32_ar)

        self.zero_config = DeepSpeedZeroConfig(pd)
        self.zero_optimization_stage = self.zero_config.stage
        self.zero_enabled = self.zero_optimization_stage > 0
        self.activation_checkpointing_config = DeepSpeedActivationCheckpointingConfig(pd)

        amp = pd.get("amp", {}) or {}
        self.amp_enabled = amp.get("enabled", False)
        self.amp_params = {k: v for k, v in amp.items() if k != "enabled"} or False

        opt = pd.get("optimizer")
        self.optimizer_name = opt.get("type") if opt else None
        if self.optimizer_name is not None and self.optimizer_name.lower() in DEEPSPEED_OPTIMIZERS:
            self.optimizer_name = self.optimizer_name.lower()
        self.optimizer_params = copy.deepcopy(opt.get("params", {})) if opt else None
        self.optimizer_legacy_fusion = opt.get("legacy_fusion", False) if opt else False

        sched = pd.get("scheduler")
        self.scheduler_name = sched.get("type") if sched else None
        self.scheduler_params = sched.get("params", {}) if sched else None

        self.flops_profiler_config = DeepSpeedFlopsProfilerConfig(pd)
        tb = pd.get("tensorboard", {}) or {}
        self.tensorboard_enabled = tb.get("enabled", False)
        self.tensorboard_output_path = tb.get("output_path", "")
        self.tensorboard_job_name = tb.get("job_name", "DeepSpeedJobName")

        self.sparse_attention = _sparse_attention_section(pd)
        self.pipeline = _pipeline_section(pd)

        pld = pd.get("progressive_layer_drop", {}) or {}
        self.pld_enabled = pld.get("enabled", False)
        self.pld_params = {"theta": pld.get("theta", 1.0), "gamma": pld.get("gamma", 0.001)} if self.pld_enabled \
            else False

        ck = pd.get("checkpoint", {}) or {}
        mode = str(ck.get("tag_validation", "Warn")).upper()
        if mode not in ValidationMode.__members__:
            raise DeepSpeedConfigError(f"Checkpoint config contains invalid tag_validation value of {mode}, "
                                       f"expecting one of {list(ValidationMode.__members__)}")
        self.checkpoint_tag_validation_enabled = ValidationMode[mode] != ValidationMode.IGNORE
        self.checkpoint_tag_validation_fail = ValidationMode[mode] == ValidationMode.FAIL
        # MI355X extension: "reference" writes ZeRO optimizer files in the reference's contiguous
        # per-group layout (zero_to_fp32.py of DeepSpeed 0.3.15 reads them); "native" (default)
        # writes this framework's per-bucket interleaved shards
        self.checkpoint_zero_format = str(ck.get("zero_format", "native")).lower()
        if self.checkpoint_zero_format not in ("native", "reference"):
            raise DeepSpeedConfigError(f"checkpoint.zero_format must be 'native' or 'reference', "
                                       f"got {self.checkpoint_zero_format!r}")

        self.aio_config = get_aio_config(pd)
        self.vocabulary_size = pd.get("vocabulary_size", None)

    # ---------------------------------------------------------------- batch triple
    def _set_batch_related_parameters(self):
        tb, mb, ga = self.train_batch_size, self.train_micro_batch_size_per_gpu, self.gradient_accumulation_steps
        ws = self.world_size
        if tb is not None and mb is not None and ga is not None:
            return
        if tb is not None and mb is not None:
            self.gradient_accumulation_steps = tb // mb // ws
        elif tb is not None and ga is not None:
            self.train_micro_batch_size_per_gpu = tb // ws // ga
        elif mb is not None and ga is not None:
            self.train_batch_size = mb * ga * ws
        elif tb is not None:
            self.gradient_accumulation_steps = 1
            self.train_micro_batch_size_per_gpu = tb // ws
        elif mb is not None:
            self.train_batch_size = mb * ws
            self.gradient_accumulation_steps = 1
        else:
            raise AssertionError("Either train_batch_size or micro_batch_per_gpu needs to be provided")

    def _batch_assertion(self):
        tb, mb, ga = self.train_batch_size, self.train_micro_batch_size_per_gpu, self.gradient_accumulation_steps
        assert tb > 0, f"Train batch size: {tb} has to be greater than 0"
        assert mb > 0, f"Micro batch size per gpu: {mb} has to be greater than 0"
        assert ga > 0, f"Gradient accumulation steps: {ga} has to be greater than 0"
        assert tb == mb * ga * self.world_size, (
            "Check batch related parameters. train_batch_size is not equal to micro_batch_per_gpu * "
            f"gradient_acc_step * world_size {tb} != {mb} * {ga} * {self.world_size}")

    def _configure_train_batch_size(self):
        self._set_batch_related_parameters()
        self._batch_assertion()

    # ---------------------------------------------------------------- checks
    def _do_sanity_check(self):
        assert self.train_micro_batch_size_per_gpu, f"DeepSpeedConfig: {TRAIN_MICRO_BATCH_SIZE_PER_GPU} is not defined"
        assert self.gradient_accumulation_steps, f"DeepSpeedConfig: {GRADIENT_ACCUMULATION_STEPS} is not defined"
        if self.zero_enabled:
            assert self.fp16_enabled, "DeepSpeedConfig: ZeRO is only supported if fp16 is enabled"
            assert self.zero_optimization_stage <= MAX_STAGE_ZERO_OPTIMIZATION
        vs = self.vocabulary_size
        if vs and vs % TENSOR_CORE_ALIGN_SIZE != 0:
            logger.warning(f"DeepSpeedConfig: vocabulary size {vs} is not aligned to {TENSOR_CORE_ALIGN_SIZE}, "
                           "may reduce matrix-core utilization.")
        if self.optimizer_params and self.optimizer_params.get(MAX_GRAD_NORM, 0) > 0:
            if self.fp16_enabled or self.zero_enabled:
                if self.global_rank == 0:
                    logger.warning(f"DeepSpeedConfig: In FP16 mode, DeepSpeed will pass {MAX_GRAD_NORM}:"
                                   f"{self.optimizer_params[MAX_GRAD_NORM]} to FP16 wrapper")
            else:
                if self.global_rank == 0:
                    logger.warning(f"DeepSpeedConfig: In FP32 mode, DeepSpeed does not permit MAX_GRAD_NORM "
                                   f"({self.optimizer_params[MAX_GRAD_NORM]}) > 0, setting to zero")
                self.optimizer_params[MAX_GRAD_NORM] = 0.0

    def print(self, name):
        logger.info("{}:".format(name))
        for arg in sorted(vars(self)):
            if arg != "_param_dict":
                logger.info("  {} {} {}".format(arg, "." * (29 - len(arg)), getattr(self, arg)))
        logger.info("  json = {}".format(json.dumps(self._param_dict, sort_keys=True, indent=4,
                                                     cls=ScientificNotationEncoder, separators=(",", ":"))))


class DeepSpeedConfigWriter:
    def __init__(self, data=None):
        self.data = data if data is not None else {}

    def add_config(self, key, value):
        self.data[key] = value

    def load_config(self, filename):
        self.data = json.load(open(filename, "r"), object_pairs_hook=dict_raise_error_on_duplicate_keys)

    def write_config(self, filename):
        with open(filename, "w") as outfile:
            json.dump(self.data, outfile)
