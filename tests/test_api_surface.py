"""SURVEY §2.8 public API surface: every reference import path resolves (through the
`deepspeed` compatibility name and natively)."""

import importlib

import pytest

PATHS = [
    ("deepspeed", ["initialize", "add_config_arguments", "init_distributed", "DeepSpeedEngine", "PipelineEngine",
                   "PipelineModule", "DeepSpeedConfig"]),
    ("deepspeed.pipe", ["PipelineModule", "LayerSpec", "TiedLayerSpec"]),
    ("deepspeed.runtime.pipe.topology", ["ProcessTopology", "PipeDataParallelTopology",
                                         "PipeModelDataParallelTopology", "PipelineParallelGrid"]),
    ("deepspeed.zero", ["Init", "GatheredParameters", "register_external_parameter", "TiledLinear",
                        "TiledLinearReturnBias", "ZeroParamStatus", "ZeroParamType"]),
    ("deepspeed.checkpointing", ["checkpoint", "configure", "model_parallel_cuda_manual_seed", "get_cuda_rng_tracker",
                                 "reset", "is_configured", "partition_activations_in_checkpoint"]),
    ("deepspeed.ops.adam", ["FusedAdam", "DeepSpeedCPUAdam"]),
    ("deepspeed.ops.lamb", ["FusedLamb"]),
    ("deepspeed.ops.transformer", ["DeepSpeedTransformerLayer", "DeepSpeedTransformerConfig"]),
    ("deepspeed.ops.sparse_attention", ["SparsityConfig", "DenseSparsityConfig", "FixedSparsityConfig",
                                        "VariableSparsityConfig", "BigBirdSparsityConfig",
                                        "BSLongformerSparsityConfig", "LocalSlidingWindowSparsityConfig",
                                        "SparseSelfAttention", "BertSparseSelfAttention", "SparseAttentionUtils",
                                        "MatMul", "Softmax"]),
    ("deepspeed.ops.aio", ["AsyncIOBuilder"]),
    ("deepspeed.runtime.fp16.onebit.adam", ["OnebitAdam"]),
    ("deepspeed.runtime.fp16.onebit.lamb", ["OnebitLamb"]),
    ("deepspeed.runtime.lr_schedules", ["LRRangeTest", "OneCycle", "WarmupLR", "WarmupDecayLR",
                                        "add_tuning_arguments"]),
    ("deepspeed.utils", ["logger", "log_dist", "RepeatingLoader"]),
    ("deepspeed.runtime.utils", ["see_memory_usage", "GradientNoiseScale", "PartitionedTensor", "partition_uniform",
                                 "partition_balanced"]),
    ("deepspeed.profiling.flops_profiler", ["FlopsProfiler", "get_model_profile"]),
    ("deepspeed.elasticity", ["compute_elastic_config"]),
    ("deepspeed.module_inject", ["replace_transformer_layer", "revert_transformer_layer", "replace_module"]),
    ("deepspeed.ops.op_builder", ["FusedAdamBuilder", "CPUAdamBuilder", "FusedLambBuilder", "TransformerBuilder",
                                  "StochasticTransformerBuilder", "SparseAttnBuilder", "AsyncIOBuilder",
                                  "UtilsBuilder"]),
    ("deepspeed.runtime.zero.stage2", ["FP16_DeepSpeedZeroOptimizer"]),
    ("deepspeed.runtime.zero.stage1", ["FP16_DeepSpeedZeroOptimizer_Stage1"]),
    ("deepspeed.runtime.zero.stage3", ["FP16_DeepSpeedZeroOptimizer_Stage3"]),
    ("deepspeed.runtime.fp16.fused_optimizer", ["FP16_Optimizer"]),
    ("deepspeed.runtime.fp16.unfused_optimizer", ["FP16_UnfusedOptimizer"]),
    ("deepspeed.runtime.fp16.loss_scaler", ["LossScaler", "DynamicLossScaler"]),
    ("deepspeed.runtime.activation_checkpointing.checkpointing", ["CheckpointFunction", "checkpoint"]),
    ("deepspeed.runtime.comm.nccl", ["NcclBackend"]),
    ("deepspeed.runtime.swap_tensor.optimizer_utils", ["OptimizerSwapper", "PipelinedOptimizerSwapper"]),
    ("deepspeed.runtime.zero.linear", ["LinearFunctionForZeroStage3", "LinearModuleForZeroStage3"]),
    ("deepspeed.runtime.zero.contiguous_memory_allocator", ["ContiguousMemoryAllocator"]),
    ("deepspeed.runtime.dataloader", ["DeepSpeedDataLoader", "RepeatingLoader"]),
    ("deepspeed.runtime.progressive_layer_drop", ["ProgressiveLayerDrop"]),
    ("deepspeed.runtime.csr_tensor", ["CSRTensor"]),
    ("deepspeed.utils.zero_to_fp32", ["convert_zero_chkpt_to_fp32_consolid_state_dict"]),
    ("deepspeed.launcher.runner", ["main", "fetch_hostfile", "parse_inclusion_exclusion"]),
    ("deepspeed.launcher.multinode_runner", ["PDSHRunner", "OpenMPIRunner", "MVAPICHRunner", "SlurmRunner"]),
    ("deepspeed.env_report", ["main"]),
    ("deepspeed.utils.timer", ["SynchronizedWallClockTimer", "ThroughputTimer"]),
]


@pytest.mark.parametrize("mod,names", PATHS, ids=[p[0] for p in PATHS])
def test_import_paths(mod, names):
    import deepspeed  # noqa: F401  (installs the alias finder)
    m = importlib.import_module(mod)
    missing = [n for n in names if not hasattr(m, n)]
    assert not missing, f"{mod} lacks {missing}"
    native = importlib.import_module(mod.replace("deepspeed", "deeperspeed_amd", 1)) if mod not in (
        "deepspeed.runtime.zero.stage2", "deepspeed.runtime.zero.stage1", "deepspeed.ops.op_builder") else m
    assert native is not None
