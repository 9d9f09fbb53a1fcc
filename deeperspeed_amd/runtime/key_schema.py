"""Named config keys and defaults, generated from the engine's own parsing tables.

The reference exposes every JSON key of the config as module-level constants
(`deepspeed/runtime/constants.py`, `runtime/zero/constants.py`, `runtime/zero/offload_constants.py`,
`runtime/swap_tensor/constants.py`, `profiling/constants.py`): for a key stem `X`, the name `X`
holds the JSON key and `X_DEFAULT` its default.  Here one table per section drives both the
parsers (runtime/config.py, runtime/zero/config.py) and those import paths, so the constants can
never drift from what the engine actually reads.
"""

from typing import Dict, List, Tuple

# (stem, json key, default); a default of _NODEF emits only the key constant
_NODEF = object()

TOP: List[Tuple[str, str, object]] = [
    ("TRAIN_BATCH_SIZE", "train_batch_size", None),
    ("TRAIN_MICRO_BATCH_SIZE_PER_GPU", "train_micro_batch_size_per_gpu", None),
    ("GRADIENT_ACCUMULATION_STEPS", "gradient_accumulation_steps", None),
    ("OPTIMIZER", "optimizer", _NODEF), ("OPTIMIZER_PARAMS", "params", _NODEF), ("TYPE", "type", _NODEF),
    ("LEGACY_FUSION", "legacy_fusion", False), ("SCHEDULER", "scheduler", _NODEF),
    ("SCHEDULER_PARAMS", "params", _NODEF), ("MAX_GRAD_NORM", "max_grad_norm", _NODEF),
    ("ZERO_ALLOW_UNTESTED_OPTIMIZER", "zero_allow_untested_optimizer", False),
    ("STEPS_PER_PRINT", "steps_per_print", 10), ("SPARSE_GRADIENTS", "sparse_gradients", False),
    ("FP16", "fp16", _NODEF), ("FP16_ENABLED", "enabled", False), ("FP16_TYPE", "type", "fp16"),
    ("FP16_LOSS_SCALE", "loss_scale", 0), ("FP16_INITIAL_SCALE_POWER", "initial_scale_power", 32),
    ("FP16_LOSS_SCALE_WINDOW", "loss_scale_window", 1000), ("FP16_HYSTERESIS", "hysteresis", 2),
    ("FP16_MIN_LOSS_SCALE", "min_loss_scale", 1), ("AMP", "amp", _NODEF), ("AMP_ENABLED", "enabled", False),
    ("GRADIENT_CLIPPING", "gradient_clipping", 0.0), ("FP32_ALLREDUCE", "fp32_allreduce", False),
    ("PRESCALE_GRADIENTS", "prescale_gradients", False),
    ("GRADIENT_PREDIVIDE_FACTOR", "gradient_predivide_factor", 1.0),
    ("DISABLE_ALLGATHER", "disable_allgather", False), ("DUMP_STATE", "dump_state", False),
    ("VOCABULARY_SIZE", "vocabulary_size", None), ("WALL_CLOCK_BREAKDOWN", "wall_clock_breakdown", False),
    ("MEMORY_BREAKDOWN", "memory_breakdown", False), ("TENSORBOARD", "tensorboard", _NODEF),
    ("TENSORBOARD_ENABLED", "enabled", False), ("TENSORBOARD_OUTPUT_PATH", "output_path", ""),
    ("TENSORBOARD_JOB_NAME", "job_name", "DeepSpeedJobName"),
    ("PROGRESSIVE_LAYER_DROP", "progressive_layer_drop", _NODEF), ("PLD_ENABLED", "enabled", False),
    ("PLD_THETA", "theta", 1.0), ("PLD_GAMMA", "gamma", 0.001), ("CHECKPOINT", "checkpoint", _NODEF),
    ("CHECKPOINT_TAG_VALIDATION", "tag_validation", "Warn"), ("CHECKPOINT_ZERO_FORMAT", "zero_format", "native"),
    ("SPARSE_ATTENTION", "sparse_attention", _NODEF), ("SPARSE_MODE", "mode", "fixed"),
    ("SPARSE_BLOCK", "block", 16), ("SPARSE_DIFFERENT_LAYOUT_PER_HEAD", "different_layout_per_head", False),
    ("SPARSE_NUM_LOCAL_BLOCKS", "num_local_blocks", 4), ("SPARSE_NUM_GLOBAL_BLOCKS", "num_global_blocks", 1),
    ("SPARSE_ATTENTION_TYPE", "attention", "bidirectional"),
    ("SPARSE_HORIZONTAL_GLOBAL_ATTENTION", "horizontal_global_attention", False),
    ("SPARSE_NUM_DIFFERENT_GLOBAL_PATTERNS", "num_different_global_patterns", 1),
    ("SPARSE_NUM_RANDOM_BLOCKS", "num_random_blocks", 0), ("SPARSE_LOCAL_WINDOW_BLOCKS", "local_window_blocks", [4]),
    ("SPARSE_GLOBAL_BLOCK_INDICES", "global_block_indices", [0]),
    ("SPARSE_GLOBAL_BLOCK_END_INDICES", "global_block_end_indices", None),
    ("SPARSE_NUM_SLIDING_WINDOW_BLOCKS", "num_sliding_window_blocks", 3),
]

ZERO: List[Tuple[str, str, object]] = [
    ("ZERO_OPTIMIZATION", "zero_optimization", _NODEF), ("ZERO_OPTIMIZATION_STAGE", "stage", 0),
    ("ZERO_OPTIMIZATION_ALLGATHER_PARTITIONS", "allgather_partitions", True),
    ("ZERO_OPTIMIZATION_REDUCE_SCATTER", "reduce_scatter", False),
    ("ZERO_OPTIMIZATION_OVERLAP_COMM", "overlap_comm", False),
    ("ZERO_OPTIMIZATION_CONTIGUOUS_GRADIENTS", "contiguous_gradients", False),
    ("ZERO_OPTIMIZATION_REDUCE_BUCKET_SIZE", "reduce_bucket_size", 500000000),
    ("ZERO_OPTIMIZATION_ALLGATHER_BUCKET_SIZE", "allgather_bucket_size", 500000000),
    ("ZERO_OPTIMIZATION_LOAD_FROM_FP32_WEIGHTS", "load_from_fp32_weights", True),
    ("ZERO_OPTIMIZATION_ELASTIC_CHECKPOINT", "elastic_checkpoint", True),
    ("ZERO_OPTIMIZATION_CPU_OFFLOAD", "cpu_offload", False),
    ("ZERO_OPTIMIZATION_CPU_OFFLOAD_PARAMS", "cpu_offload_params", False),
    ("ZERO_OPTIMIZATION_CPU_OFFLOAD_USE_PIN_MEMORY", "cpu_offload_use_pin_memory", False),
    ("ZERO_OPTIMIZATION_OFFLOAD_PARAM", "offload_param", None),
    ("ZERO_OPTIMIZATION_OFFLOAD_OPTIMIZER", "offload_optimizer", None),
    ("ZERO_OPTIMIZATION_SUB_GROUP_SIZE", "sub_group_size", 1000000000000),
    ("ZERO_OPTIMIZATION_MAX_LIVE_PARAMETERS", "stage3_max_live_parameters", 1000000000),
    ("ZERO_OPTIMIZATION_MAX_REUSE_DISTANCE", "stage3_max_reuse_distance", 1000000000),
    ("ZERO_OPTIMIZATION_PREFETCH_BUCKET_SIZE", "stage3_prefetch_bucket_size", 50000000),
    ("ZERO_OPTIMIZATION_PARAM_PERSISTENCE_THRESHOLD", "stage3_param_persistence_threshold", 100000),
    ("ZERO_OPTIMIZATION_GATHER_FP16_WEIGHTS_ON_MODEL_SAVE", "stage3_gather_fp16_weights_on_model_save", False),
]

OFFLOAD: List[Tuple[str, str, object]] = [
    ("OFFLOAD_PARAM", "offload_param", _NODEF), ("OFFLOAD_PARAM_DEVICE", "device", "cpu"),
    ("OFFLOAD_PARAM_NVME_PATH", "nvme_path", None), ("OFFLOAD_PARAM_BUFFER_COUNT", "buffer_count", 5),
    ("OFFLOAD_PARAM_BUFFER_SIZE", "buffer_size", 100000000), ("OFFLOAD_PARAM_MAX_IN_CPU", "max_in_cpu", 1000000000),
    ("OFFLOAD_PARAM_PIN_MEMORY", "pin_memory", False), ("OFFLOAD_OPTIMIZER", "offload_optimizer", _NODEF),
    ("OFFLOAD_OPTIMIZER_DEVICE", "device", "cpu"), ("OFFLOAD_OPTIMIZER_NVME_PATH", "nvme_path", None),
    ("OFFLOAD_OPTIMIZER_BUFFER_COUNT", "buffer_count", 4), ("OFFLOAD_OPTIMIZER_PIN_MEMORY", "pin_memory", False),
    ("OFFLOAD_OPTIMIZER_PIPELINE_READ", "pipeline_read", False),
    ("OFFLOAD_OPTIMIZER_PIPELINE_WRITE", "pipeline_write", False),
    ("OFFLOAD_OPTIMIZER_PIPELINE", "pipeline", _NODEF), ("OFFLOAD_OPTIMIZER_FAST_INIT", "fast_init", False),
]

AIO: List[Tuple[str, str, object]] = [
    ("AIO", "aio", _NODEF), ("AIO_BLOCK_SIZE", "block_size", 1048576), ("AIO_QUEUE_DEPTH", "queue_depth", 8),
    ("AIO_THREAD_COUNT", "thread_count", 1), ("AIO_SINGLE_SUBMIT", "single_submit", False),
    ("AIO_OVERLAP_EVENTS", "overlap_events", True),
]

FLOPS_PROFILER: List[Tuple[str, str, object]] = [
    ("FLOPS_PROFILER", "flops_profiler", _NODEF), ("FLOPS_PROFILER_ENABLED", "enabled", False),
    ("FLOPS_PROFILER_PROFILE_STEP", "profile_step", 1), ("FLOPS_PROFILER_MODULE_DEPTH", "module_depth", -1),
    ("FLOPS_PROFILER_TOP_MODULES", "top_modules", 3), ("FLOPS_PROFILER_DETAILED", "detailed", True),
]


def export(table) -> Dict[str, object]:
    """{STEM: key, STEM_DEFAULT: default, <section>_FORMAT: short doc} for a section table."""
    out: Dict[str, object] = {}
    for stem, key, default in table:
        out[stem] = key
        if default is not _NODEF:
            out[stem + "_DEFAULT"] = default
    head = table[0][0]
    keys = ", ".join(f'"{k}"' for _, k, d in table[1:] if d is not _NODEF)
    out[head + "_FORMAT"] = f'"{table[0][1]}": {{{keys}}}'
    return out


def defaults(table) -> Dict[str, object]:
    """{json key: default} of a section (the parsers' default dicts)."""
    return {key: d for _, key, d in table[1:] if d is not _NODEF}
