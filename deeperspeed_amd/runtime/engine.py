"""DeepSpeedEngine: the training loop wrapper returned by `deepspeed.initialize()`.

Reference parity: deepspeed/runtime/engine.py:102-1915 (config accessors, distributed model
setup, optimizer/scheduler selection, forward/backward/step with gradient accumulation,
gradient clipping, overflow-skip accounting, progress/tensorboard reporting, checkpoint
save/load in the same on-disk layout, fp16 model export) plus the DeeperSpeed additions:
`register_forward_hook(layers_to_hook)` / `layer_outputs` (engine.py:222-254) and the
`store_gradients[_cpu]` gradient snapshot (engine.py:139-141,1156-1161).

MI355X design: every mixed-precision / ZeRO mode runs on the flat-arena optimizers
(runtime/zero/*) whose gradient reductions are issued from backward hooks on RCCL's stream;
the engine never calls `torch.cuda.synchronize()` on the hot path.
"""

from __future__ import annotations

import hashlib
import os
import re
import shutil
from collections import OrderedDict

import torch
import torch.distributed as dist
from torch.nn.modules import Module

from ..ops import linear as _linear_ops
from ..ops import wgrad_batch as _wgrad_batch
from ..ops.adam.fused_adam import FusedAdam
from ..utils.distributed import init_distributed
from ..utils import comm
from ..utils.logging import log_dist, logger
from ..utils.timer import SynchronizedWallClockTimer, ThroughputTimer
from ..version import __version__
from . import lr_schedules
from .config import (ADAM_OPTIMIZER, ADAM_W_MODE, ADAM_W_MODE_DEFAULT, ADAMW_OPTIMIZER, DEEPSPEED_OPTIMIZERS,
                     LAMB_OPTIMIZER, MAX_GRAD_NORM, ONEBIT_ADAM_OPTIMIZER, ONEBIT_LAMB_OPTIMIZER, TORCH_ADAM_PARAM,
                     DeepSpeedConfig)
from .dataloader import DeepSpeedDataLoader
from .utils import clip_grad_norm_, see_memory_usage
from .zero.config import ZERO_OPTIMIZATION_GRADIENTS, ZERO_OPTIMIZATION_OPTIMIZER_STATES, ZERO_OPTIMIZATION_WEIGHTS

MEMORY_OPT_ALLREDUCE_SIZE = 500000000


def split_half_float_double_csr(tensors):
    buckets = OrderedDict()
    for t in tensors:
        key = (t.dtype, t.layout)
        buckets.setdefault(key, []).append(t)
    return list(buckets.values())


def _initialize_parameter_parallel_groups(parameter_parallel_size=None):
    data_parallel_size = int(dist.get_world_size())
    parameter_parallel_size = parameter_parallel_size or data_parallel_size
    assert data_parallel_size % parameter_parallel_size == 0
    rank = dist.get_rank()
    my_group = None
    for i in range(data_parallel_size // parameter_parallel_size):
        ranks = range(i * parameter_parallel_size, (i + 1) * parameter_parallel_size)
        group = dist.new_group(ranks)
        if rank in ranks:
            my_group = group
    return my_group


class DeepSpeedEngine(Module):
    r"""DeepSpeed engine for training."""

    def __init__(self, args, model, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
                 mpu=None, dist_init_required=None, collate_fn=None, config_params=None, dont_change_device=False):
        super().__init__()
        self.dont_change_device = dont_change_device
        self.client_optimizer = optimizer
        self.client_model_parameters = model_parameters
        self.client_lr_scheduler = lr_scheduler
        self.training_data = training_data
        self.collate_fn = collate_fn
        self.mpu = mpu
        self.data_parallel_group = None
        self.global_steps = 0
        self.global_samples = 0
        self.micro_steps = 0
        self.skipped_steps = 0
        self.gradient_average = True
        self.warn_unscaled_loss = True
        self.config_params = config_params
        self.loaded_checkpoint_mp_world_size = None
        self.loaded_checkpoint_dp_world_size = None
        self.enable_backward_allreduce = True
        self.progressive_layer_drop = None
        self.dist_backend = "nccl"
        self.store_gradients = False
        self.store_gradients_cpu = True
        self.stored_gradients = None
        self.summary_writer = None
        self.flops_profiler = None

        if dist_init_required is None:
            dist_init_required = not dist.is_initialized()
        if dist_init_required is False:
            assert dist.is_initialized(), ("Torch distributed not initialized. Please set dist_init_required to "
                                           "True or initialize before calling deepspeed.initialize()")
        else:
            init_distributed(dist_backend=self.dist_backend)

        self._do_args_sanity_check(args)
        self._configure_with_arguments(args, mpu)
        if mpu is not None:
            assert not self.elasticity_enabled(), "Elasticity is not currently supported with model parallelism."
        self._set_distributed_vars()
        if self.tensorboard_enabled() and self.global_rank == 0:
            self.summary_writer = self.get_summary_writer()

        self._configure_distributed_model(model)
        self.timers = SynchronizedWallClockTimer()
        self.tput_timer = ThroughputTimer(batch_size=self.train_micro_batch_size_per_gpu(),
                                          num_workers=self.dp_world_size, steps_per_output=self.steps_per_print(),
                                          monitor_memory=False)
        self.training_dataloader = self.deepspeed_io(training_data) if training_data else None

        self.optimizer = None
        self.amp = None  # runtime/amp.py AmpState when "amp": {"enabled": true}
        self.basic_optimizer = None
        self.lr_scheduler = None
        if model_parameters or optimizer:
            self._configure_optimizer(optimizer, model_parameters)
            self._configure_lr_scheduler(lr_scheduler)
            self._report_progress(0)
        # weight gradients may wait for the end of backward only where no gradient hook reads them
        # during it: no ZeRO stage, no bucket hooks of a flat-arena optimizer, no overlapped step;
        # then equal layers' weight gradients run as batched GEMMs (ops/wgrad_batch.py) with their
        # .grad bound to persistent stacks the fp16 optimizer zeroes in place
        from .fp16.unfused_optimizer import FP16_UnfusedOptimizer
        self._defer_wgrad = (isinstance(self.optimizer, FP16_UnfusedOptimizer) and self.device.type == "cuda"
                             and not self.zero_optimization() and getattr(self.optimizer, "_overlap", None) is None
                             and _wgrad_batch.ENABLED)
        _wgrad_batch.enable(self._defer_wgrad)
        if self._defer_wgrad:
            _wgrad_batch.bind_grad_stacks(self.module.parameters())

        self.csr_tensor_module_names = set()
        if self.sparse_gradients_enabled():
            for name, module in self.module.named_modules():
                if isinstance(module, torch.nn.Embedding):
                    self.csr_tensor_module_names.add(name + ".weight")
                    logger.info("Will convert {} to sparse (csr) tensor during training".format(name))

        self.save_non_zero_checkpoint = False
        self.save_zero_checkpoint = False
        self._configure_checkpointing(dist_init_required)
        if self.pld_enabled():
            self.progressive_layer_drop = self._configure_progressive_layer_drop()
        if self.global_rank == 0:
            self._config.print("DeepSpeedEngine configuration")

        from ..ops.native import _cpu_flatten
        self.flatten, self.unflatten = _cpu_flatten()

        # DeeperSpeed forward-activation capture
        self.layer_outputs, self.layers_to_hook, self.hooks = {}, [], []
        self.layer_name_pattern = "transformerlayer"
        self.register_forward_hook(layers_to_hook=self.layers_to_hook)

    # ------------------------------------------------------------------ DeeperSpeed hooks
    def register_forward_hook(self, layers_to_hook, layer_name_pattern: str = "transformerlayer"):
        """Capture forward outputs of layers whose class name matches `layer_name_pattern`
        (case-insensitive) into `self.layer_outputs` (moved to host).  Layers exposing
        `layer_number` are keyed by it and filtered by `layers_to_hook` ("all" or a list)."""
        self.layer_name_pattern = re.compile(layer_name_pattern, re.IGNORECASE)
        self.layers_to_hook = layers_to_hook
        for h in self.hooks:
            h.remove()
        self.hooks = []
        if not layers_to_hook:
            return

        def hook_fn(module, inputs, output):
            if hasattr(module, "layer_number"):
                key = module.layer_number
                if self.layers_to_hook != "all" and int(key) not in self.layers_to_hook:
                    return
            else:
                key = module.__class__.__name__
            outs = output if isinstance(output, (list, tuple)) else [output]
            self.layer_outputs[key] = [o.detach().cpu() if torch.is_tensor(o) else o for o in outs]

        def visit(net):
            for _, layer in net._modules.items():
                if layer is None:
                    continue
                if isinstance(layer, torch.nn.Sequential) or isinstance(layer, torch.nn.ModuleList):
                    visit(layer)
                elif self.layer_name_pattern.search(layer.__class__.__name__.lower()):
                    self.hooks.append(layer.register_forward_hook(hook_fn))
                else:
                    visit(layer)

        visit(self.module)

    # ------------------------------------------------------------------ config accessors
    def get_batch_info(self):
        return self.train_batch_size(), self.train_micro_batch_size_per_gpu(), self.gradient_accumulation_steps()

    def elasticity_enabled(self):
        return self._config.elasticity_enabled

    def pld_enabled(self):
        return self._config.pld_enabled

    def pld_params(self):
        return self._config.pld_params

    def pld_theta(self):
        return self.pld_params()["theta"]

    def pld_gamma(self):
        return self.pld_params()["gamma"]

    def tensorboard_enabled(self):
        return self._config.tensorboard_enabled

    def tensorboard_output_path(self):
        return self._config.tensorboard_output_path

    def tensorboard_job_name(self):
        return self._config.tensorboard_job_name

    def get_summary_writer(self, name="DeepSpeedJobName", base=os.path.join(os.path.expanduser("~"), "tensorboard")):
        if self.tensorboard_output_path():
            base_dir = self.tensorboard_output_path()
            job_name = self.tensorboard_job_name()
            log_dir = os.path.join(base_dir, job_name)
        else:
            job_name = self.tensorboard_job_name() or name
            infra = os.environ.get("DLWS_JOB_ID") or os.environ.get("DLTS_JOB_ID") or "unknown-job-id"
            log_dir = os.path.join(base, infra, "logs", job_name)
        os.makedirs(log_dir, exist_ok=True)
        try:
            from torch.utils.tensorboard import SummaryWriter
        except Exception:  # tensorboard not installed: native event-file writer
            from ..utils.tb_writer import EventFileWriter
            return EventFileWriter(log_dir)
        return SummaryWriter(log_dir=log_dir)

    def wall_clock_breakdown(self):
        return self._config.wall_clock_breakdown

    def flops_profiler_enabled(self):
        return self._config.flops_profiler_config.enabled

    def flops_profiler_profile_step(self):
        return self._config.flops_profiler_config.profile_step

    def flops_profiler_module_depth(self):
        return self._config.flops_profiler_config.module_depth

    def flops_profiler_top_modules(self):
        return self._config.flops_profiler_config.top_modules

    def flops_profiler_detailed(self):
        return self._config.flops_profiler_config.detailed

    def memory_breakdown(self):
        return self._config.memory_breakdown

    def sparse_gradients_enabled(self):
        return self._config.sparse_gradients_enabled

    def train_batch_size(self):
        return self._config.train_batch_size

    def train_micro_batch_size_per_gpu(self):
        return self._config.train_micro_batch_size_per_gpu

    def optimizer_name(self):
        return self.client_optimizer.__class__.__name__ if self.client_optimizer else self._config.optimizer_name

    def optimizer_params(self):
        return self._config.optimizer_params

    def optimizer_legacy_fusion(self):
        return self._config.optimizer_legacy_fusion

    def scheduler_name(self):
        return self._config.scheduler_name

    def scheduler_params(self):
        return self._config.scheduler_params

    def zero_optimization(self):
        return self._config.zero_enabled

    def zero_allow_untested_optimizer(self):
        return self._config.zero_allow_untested_optimizer

    def zero_reduce_scatter(self):
        return self._config.zero_config.reduce_scatter

    def zero_overlap_comm(self):
        return self._config.zero_config.overlap_comm

    def zero_offload_optimizer(self):
        return self._config.zero_config.offload_optimizer

    def zero_offload_param(self):
        return self._config.zero_config.offload_param

    def zero_cpu_offload(self):
        return self._config.zero_config.offload_optimizer is not None

    def zero_sub_group_size(self):
        return self._config.zero_config.sub_group_size

    def zero_optimization_stage(self):
        return self._config.zero_optimization_stage

    def zero_reduce_bucket_size(self):
        return self._config.zero_config.reduce_bucket_size

    def zero_allgather_bucket_size(self):
        return self._config.zero_config.allgather_bucket_size

    def zero_optimization_partition_gradients(self):
        return self.zero_optimization_stage() >= ZERO_OPTIMIZATION_GRADIENTS

    def zero_optimization_partition_weights(self):
        return self.zero_optimization_stage() >= ZERO_OPTIMIZATION_WEIGHTS

    def zero_contiguous_gradients(self):
        return self._config.zero_config.contiguous_gradients

    def zero_load_from_fp32_weights(self):
        return self._config.zero_config.load_from_fp32_weights

    def zero_elastic_checkpoint(self):
        return self._config.zero_config.elastic_checkpoint

    def zero_max_live_parameters(self):
        return self._config.zero_config.stage3_max_live_parameters

    def zero_max_reuse_distance(self):
        return self._config.zero_config.stage3_max_reuse_distance

    def zero_prefetch_bucket_size(self):
        return self._config.zero_config.stage3_prefetch_bucket_size

    def zero_param_persistence_threshold(self):
        return self._config.zero_config.stage3_param_persistence_threshold

    def zero_gather_fp16_weights_on_model_save(self):
        return self._config.zero_config.stage3_gather_fp16_weights_on_model_save

    def fp16_enabled(self):
        return self._config.fp16_enabled

    def bfloat16_enabled(self):
        return self._config.bfloat16_enabled

    def precision(self):
        return self._config.precision

    def amp_enabled(self):
        return self._config.amp_enabled

    def amp_params(self):
        return self._config.amp_params

    def loss_scale(self):
        return self._config.loss_scale

    def gradient_accumulation_steps(self):
        return self._config.gradient_accumulation_steps

    def allreduce_always_fp32(self):
        return self._config.allreduce_always_fp32

    def postscale_gradients(self):
        return not self._config.prescale_gradients

    def gradient_predivide_factor(self):
        return self._config.gradient_predivide_factor

    def steps_per_print(self):
        return self._config.steps_per_print

    def zero_allgather_partitions(self):
        return self._config.zero_config.allgather_partitions

    def dump_state(self):
        return self._config.dump_state

    def gradient_clipping(self):
        return self._config.gradient_clipping

    def dynamic_loss_scale(self):
        return self._config.loss_scale == 0

    def initial_dynamic_scale(self):
        return self._config.initial_dynamic_scale

    def dynamic_loss_scale_args(self):
        return self._config.dynamic_loss_scale_args

    def swap_tensor_config(self):
        return self._config.aio_config

    def aio_config(self):
        return self._config.aio_config

    # ------------------------------------------------------------------ setup
    def _configure_lr_scheduler(self, client_lr_scheduler):
        lr_scheduler = self._scheduler_from_config(self.optimizer)
        if lr_scheduler:
            if self.global_rank == 0:
                logger.info(f"DeepSpeed using configured LR scheduler = {self.scheduler_name()}")
            self.lr_scheduler = lr_scheduler
        else:
            if self.global_rank == 0:
                logger.info("DeepSpeed using client LR scheduler")
            self.lr_scheduler = client_lr_scheduler
        log_dist(f"DeepSpeed LR Scheduler = {self.lr_scheduler}", ranks=[0])

    def _configure_checkpointing(self, dist_init_required):
        dp_rank = self.global_rank
        if self.mpu:
            dp_rank = self.mpu.get_data_parallel_rank()
        self.save_non_zero_checkpoint = (dp_rank == 0) or self.zero_optimization_partition_weights()
        if self.zero_optimization():
            param_rank = dist.get_rank(group=self.optimizer.dp_group) if dist.is_initialized() else 0
            self.save_zero_checkpoint = param_rank == dp_rank

    def _scheduler_from_config(self, optimizer):
        name = self.scheduler_name()
        if name is None:
            return None
        if hasattr(lr_schedules, name):
            sched = getattr(lr_schedules, name)
        else:
            assert hasattr(torch.optim.lr_scheduler, name), f"DeepSpeed does not recognize LR scheduler {name}"
            sched = getattr(torch.optim.lr_scheduler, name)
        base = lr_schedules.get_torch_optimizer(optimizer)
        return sched(base, **self.scheduler_params())

    def _set_distributed_vars(self):
        if torch.cuda.is_available():
            self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(self.local_rank % max(1, torch.cuda.device_count()))
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
            self.device = torch.device("cpu")
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.global_rank = dist.get_rank() if dist.is_initialized() else 0

    def _configure_with_arguments(self, args, mpu):
        self.local_rank = int(os.environ.get("LOCAL_RANK", getattr(args, "local_rank", 0) or 0))
        config_file = getattr(args, "deepspeed_config", None) if args is not None else None
        if config_file is None and args is not None:
            config_file = getattr(args, "deepscale_config", None)
        self._config = DeepSpeedConfig(config_file, mpu, param_dict=self.config_params)

    def _do_args_sanity_check(self, args):
        if args is not None and hasattr(args, "deepscale_config") and args.deepscale_config is not None:
            logger.warning("************ --deepscale_config is deprecated, please use --deepspeed_config ************")
            if hasattr(args, "deepspeed_config"):
                assert args.deepspeed_config is None, \
                    "Not sure how to proceed, we were given both a deepscale_config and deepspeed_config"
            args.deepspeed_config = args.deepscale_config
        if self.config_params is None:
            assert args is not None and getattr(args, "deepspeed_config", None) is not None, \
                "DeepSpeed requires --deepspeed_config to specify configuration file"
            assert os.path.isfile(args.deepspeed_config), \
                "DeepSpeed configuration file: {} is not an existing file".format(args.deepspeed_config)

    def _is_supported_optimizer(self, optimizer_name):
        return optimizer_name in DEEPSPEED_OPTIMIZERS or getattr(torch.optim, optimizer_name, None) is not None

    def _broadcast_model(self):
        def is_replicated(p):
            return getattr(p, "ds_tensor", None) is None
        src = self._dp_src_rank()
        for p in self.module.parameters():
            if torch.is_tensor(p) and is_replicated(p) and p.numel() > 0:
                if self.allreduce_always_fp32() and p.dtype != torch.float32:
                    t = p.data.float()
                    dist.broadcast(t, src, group=self.data_parallel_group)
                    p.data.copy_(t)
                else:
                    dist.broadcast(p.data, src, group=self.data_parallel_group)

    def _dp_src_rank(self):
        if self.mpu is not None and hasattr(self.mpu, "get_data_parallel_src_rank"):
            return self.mpu.get_data_parallel_src_rank()
        if self.mpu is not None:
            ranks = dist.get_process_group_ranks(self.data_parallel_group) \
                if hasattr(dist, "get_process_group_ranks") else None
            return ranks[0] if ranks else 0
        return 0

    def _configure_distributed_model(self, model):
        self.module = model
        if self.fp16_enabled():
            self.module.to(self.precision())
        if not self.dont_change_device:
            self.module.to(self.device)
        if self.mpu is None:
            self.data_parallel_group = _initialize_parameter_parallel_groups() if dist.is_initialized() else None
            self.dp_world_size = dist.get_world_size() if dist.is_initialized() else 1
            self.mp_world_size = 1
        else:
            self.data_parallel_group = self.mpu.get_data_parallel_group()
            self.dp_world_size = self.mpu.get_data_parallel_world_size()
            self.mp_world_size = self.mpu.get_model_parallel_world_size()
        # (amp included: the reference broadcasts after amp.initialize, REF engine.py:693-694)
        if dist.is_initialized() and self.dp_world_size > 1 and \
                os.environ.get("DSA_SKIP_MODEL_BROADCAST", "0") != "1":
            self._broadcast_model()

    # ------------------------------------------------------------------ optimizer
    def _configure_optimizer(self, client_optimizer, model_parameters):
        if client_optimizer is not None:
            if isinstance(client_optimizer, torch.optim.Optimizer) or hasattr(client_optimizer, "param_groups"):
                basic_optimizer = client_optimizer
            else:  # callable taking params
                basic_optimizer = client_optimizer(model_parameters)
            if self.global_rank == 0:
                logger.info("Using client Optimizer as basic optimizer")
        else:
            basic_optimizer = self._configure_basic_optimizer(model_parameters)
            if self.global_rank == 0:
                logger.info("Using DeepSpeed Optimizer param name {} as basic optimizer".format(
                    self.optimizer_name()))
        self.basic_optimizer = basic_optimizer
        if self.global_rank == 0:
            logger.info("DeepSpeed Basic Optimizer = {}".format(basic_optimizer.__class__.__name__))

        name = (self.optimizer_name() or "").lower()
        if name in (ONEBIT_ADAM_OPTIMIZER, ONEBIT_LAMB_OPTIMIZER) and self.zero_optimization():
            raise AssertionError("1-bit optimizers are not compatible with ZeRO")
        if self.zero_optimization():
            assert not self.amp_enabled(), ("Amp and ZeRO are not currently compatible: use the bf16 / fp16 "
                                            "config blocks (\"fp16\": {\"enabled\": true, \"type\": \"bfloat16\"})")
            self.optimizer = self._configure_zero_optimizer(basic_optimizer)
        elif self.amp_enabled():
            assert not self.fp16_enabled(), "Cannot enable both amp with (legacy) fp16 mode"
            from .amp import AmpState
            self.amp = AmpState(self.amp_params() or {}, self.device)
            log_dist(f"amp: fp32 master parameters, forward under autocast({self.amp.dtype}), "
                     f"opt_level {self.amp.opt_level}, loss scaling "
                     f"{'dynamic' if self.amp.scaler is not None else 'off'}", ranks=[0])
            self.optimizer = basic_optimizer
        elif self.fp16_enabled():
            self.optimizer = self._configure_fp16_optimizer(basic_optimizer)
        else:
            self.optimizer = basic_optimizer
        log_dist("DeepSpeed Final Optimizer = {}".format(self.optimizer.__class__.__name__), ranks=[0])

    def _configure_basic_optimizer(self, model_parameters):
        params = dict(self.optimizer_params() or {})
        params.pop(MAX_GRAD_NORM, None)
        name = (self.optimizer_name() or "adam").lower() if self._config.optimizer_name else "adam"
        if self._config.optimizer_name is None:
            raise AssertionError("No optimizer in the DeepSpeed config and no client optimizer given")
        if name in (ADAM_OPTIMIZER, ADAMW_OPTIMIZER):
            torch_adam = params.pop(TORCH_ADAM_PARAM, False)
            adam_w_mode = params.pop(ADAM_W_MODE, ADAM_W_MODE_DEFAULT)
            if name == ADAMW_OPTIMIZER:
                adam_w_mode = True
            offload = self.zero_offload_optimizer()
            if torch_adam:
                cls = torch.optim.AdamW if adam_w_mode else torch.optim.Adam
                return cls(model_parameters, **params)
            if offload is not None and offload.get("states", "all") == "all":
                from ..ops.adam.cpu_adam import DeepSpeedCPUAdam
                return DeepSpeedCPUAdam(model_parameters, adamw_mode=adam_w_mode, **params)
            return FusedAdam(model_parameters, adam_w_mode=adam_w_mode, **params)
        if name == LAMB_OPTIMIZER:
            from ..ops.lamb.fused_lamb import FusedLamb
            return FusedLamb(model_parameters, **params)
        if name == ONEBIT_ADAM_OPTIMIZER:
            from .fp16.onebit.adam import OnebitAdam
            return OnebitAdam(model_parameters, self, **params)
        if name == ONEBIT_LAMB_OPTIMIZER:
            from .fp16.onebit.lamb import OnebitLamb
            return OnebitLamb(model_parameters, self, **params)
        torch_name = self._config.optimizer_name
        cls = getattr(torch.optim, torch_name, None) or getattr(torch.optim, torch_name.capitalize(), None)
        if cls is None:
            for attr in dir(torch.optim):
                if attr.lower() == name:
                    cls = getattr(torch.optim, attr)
        assert cls is not None, f"Unknown optimizer {torch_name}"
        return cls(model_parameters, **params)

    def _dynamic_args(self):
        a = dict(self.dynamic_loss_scale_args() or {})
        return a

    def _configure_fp16_optimizer(self, optimizer):
        from .zero.stage_1_and_2 import DeepSpeedZeroOptimizer
        self._resolve_bucket_sizes(self._config.zero_config)
        dynamic = self.dynamic_loss_scale() and not self.bfloat16_enabled()
        if getattr(optimizer, "requires_per_param_masters", False):
            # per-tensor optimizer math (LAMB trust ratio): reference engine.py picks
            # FP16_UnfusedOptimizer for non-fused-Adam optimizers
            from .fp16.unfused_optimizer import FP16_UnfusedOptimizer
            return FP16_UnfusedOptimizer(optimizer, static_loss_scale=self.loss_scale() or 1.0,
                                         dynamic_loss_scale=dynamic, dynamic_loss_args=self._dynamic_args(),
                                         mpu=self.mpu, clip_grad=self.gradient_clipping(),
                                         verbose=self.global_rank == 0,
                                         overlap_step=bool(getattr(self._config.zero_config, "overlap_step", False)),
                                         module=self.module)
        return DeepSpeedZeroOptimizer(optimizer, stage=0, dp_process_group=self.data_parallel_group, mpu=self.mpu,
                                      clip_grad=self.gradient_clipping(), static_loss_scale=self.loss_scale() or 1.0,
                                      dynamic_loss_scale=dynamic, dynamic_loss_args=self._dynamic_args(),
                                      reduce_bucket_size=self.zero_reduce_bucket_size(),
                                      fp32_reduce=self.allreduce_always_fp32(),
                                      gradient_accumulation_steps=self.gradient_accumulation_steps(),
                                      timers=self.timers if self.wall_clock_breakdown() else None,
                                      verbose=self.global_rank == 0)

    def _offload_with_aio(self, off):
        """The NVMe swapper needs the `aio` section next to the offload settings."""
        if off is None:
            return None
        off = dict(off)
        aio = getattr(self._config, "aio_config", None)
        if aio:
            off["aio"] = dict(aio)
        return off

    def _resolve_bucket_sizes(self, zc):
        """'auto' ZeRO bucket sizes from the data-parallel world (runtime/comm/bucket_sizing.py)."""
        from .comm import bucket_sizing
        world = comm.world_size(self.data_parallel_group)
        esize = 2 if (self.fp16_enabled() or self.bfloat16_enabled()) else 4
        for key, scale in (("reduce_bucket_size", 1.0), ("allgather_bucket_size", 1.0),
                           ("stage3_prefetch_bucket_size", 1.0)):
            v = getattr(zc, key)
            if isinstance(v, str):
                setattr(zc, key, bucket_sizing.resolve(v, world, esize, scale))
                if self.global_rank == 0:
                    logger.info(f"ZeRO {key}=auto -> {getattr(zc, key):,} elements for {world} data-parallel ranks")

    def _configure_zero_optimizer(self, optimizer):
        stage = self.zero_optimization_stage()
        zc = self._config.zero_config
        self._resolve_bucket_sizes(zc)
        dynamic = self.dynamic_loss_scale() and not self.bfloat16_enabled()
        common = dict(dp_process_group=self.data_parallel_group, mpu=self.mpu, clip_grad=self.gradient_clipping(),
                      static_loss_scale=self.loss_scale() or 1.0, dynamic_loss_scale=dynamic,
                      dynamic_loss_args=self._dynamic_args(), fp32_reduce=self.allreduce_always_fp32(),
                      gradient_predivide_factor=self.gradient_predivide_factor(),
                      gradient_accumulation_steps=self.gradient_accumulation_steps(),
                      offload_optimizer=self._offload_with_aio(zc.offload_optimizer),
                      compact_master=bool(zc.compact_master),
                      timers=self.timers if self.wall_clock_breakdown() else None, verbose=self.global_rank == 0)
        if stage in (ZERO_OPTIMIZATION_OPTIMIZER_STATES, ZERO_OPTIMIZATION_GRADIENTS):
            from .zero.stage_1_and_2 import DeepSpeedZeroOptimizer
            return DeepSpeedZeroOptimizer(optimizer, stage=stage, reduce_bucket_size=zc.reduce_bucket_size,
                                          allgather_bucket_size=zc.allgather_bucket_size, overlap_comm=zc.overlap_comm,
                                          reduce_scatter=zc.reduce_scatter, resident_grads=bool(zc.resident_grads),
                                          sub_group_size=zc.sub_group_size, **common)
        if stage == ZERO_OPTIMIZATION_WEIGHTS:
            from .zero.stage3 import DeepSpeedZeroOptimizer_Stage3
            unit = zc.stage3_unit_max_numel
            return DeepSpeedZeroOptimizer_Stage3(self.module, optimizer,
                                                 force_sharded=bool(zc.stage3_force_sharded),
                                                 resident_grads=bool(zc.resident_grads),
                                                 grad_accum_dtype=zc.grad_accum_dtype,
                                                 reduce_scatter=zc.reduce_scatter,
                                                 reduce_bucket_size=zc.reduce_bucket_size,
                                                 prefetch_bucket_size=zc.stage3_prefetch_bucket_size,
                                                 max_live_parameters=zc.stage3_max_live_parameters,
                                                 max_reuse_distance=zc.stage3_max_reuse_distance,
                                                 param_persistence_threshold=zc.stage3_param_persistence_threshold,
                                                 unit_max_numel=unit, offload_param=zc.offload_param,
                                                 overlap_comm=zc.overlap_comm, sub_group_size=zc.sub_group_size,
                                                 overlap_step=bool(getattr(zc, "overlap_step", False)), **common)
        raise NotImplementedError("ZeRO stage {} not implemented".format(stage))

    def _configure_progressive_layer_drop(self):
        from .progressive_layer_drop import ProgressiveLayerDrop
        return ProgressiveLayerDrop(theta=self.pld_theta(), gamma=self.pld_gamma())

    def deepspeed_io(self, dataset, batch_size=None, route="train", pin_memory=True, data_sampler=None,
                     collate_fn=None, num_local_io_workers=None):
        if not isinstance(dataset, torch.utils.data.Dataset):
            raise ValueError("Training data must be a torch Dataset")
        if data_sampler is None and (route == "predict" or route == "eval"):
            data_sampler = torch.utils.data.SequentialSampler(dataset)
        if batch_size is None:
            batch_size = self.train_micro_batch_size_per_gpu()
        if collate_fn is None:
            collate_fn = self.collate_fn
        deepspeed_io_timer = self.tput_timer if route == "train" else None
        dp_world = self.mpu.get_data_parallel_world_size() if self.mpu else (
            dist.get_world_size() if dist.is_initialized() else 1)
        dp_rank = self.mpu.get_data_parallel_rank() if self.mpu else (dist.get_rank() if dist.is_initialized() else 0)
        return DeepSpeedDataLoader(dataset=dataset, batch_size=batch_size, pin_memory=pin_memory and
                                   torch.cuda.is_available(), collate_fn=collate_fn, local_rank=self.local_rank,
                                   tput_timer=deepspeed_io_timer, num_local_io_workers=num_local_io_workers or 0,
                                   data_sampler=data_sampler, data_parallel_world_size=dp_world,
                                   data_parallel_rank=dp_rank)

    # ------------------------------------------------------------------ train / eval
    def train(self, mode=True):
        self.warn_unscaled_loss = True
        self.module.train(mode)
        return self

    def eval(self):
        self.warn_unscaled_loss = True
        self.module.train(False)
        return self

    def _scale_loss(self, prescaled_loss):
        if isinstance(prescaled_loss, torch.Tensor):
            return prescaled_loss / self.gradient_accumulation_steps()
        if isinstance(prescaled_loss, (tuple, list)):
            return type(prescaled_loss)(l / self.gradient_accumulation_steps() if isinstance(l, torch.Tensor) else l
                                        for l in prescaled_loss)
        if self.warn_unscaled_loss:
            logger.warning(f"DeepSpeed unable to scale loss because of type: {type(prescaled_loss)}")
            self.warn_unscaled_loss = False
        return prescaled_loss

    def forward(self, *inputs, **kwargs):
        with comm.trace_range("engine.forward"):
            return self._forward_impl(*inputs, **kwargs)

    def _forward_impl(self, *inputs, **kwargs):
        if self.flops_profiler_enabled() and self.global_steps == self.flops_profiler_profile_step() and \
                self.global_rank == 0:
            from ..profiling.flops_profiler import FlopsProfiler
            self.flops_profiler = FlopsProfiler(self.module)
            self.flops_profiler.start_profile(ignore_list=None)
        if self.module.training and self.progressive_layer_drop:
            kwargs.update(self.progressive_layer_drop.get_state())
        if self.wall_clock_breakdown():
            self.timers("forward_microstep").start()
            self.timers("forward").start()
        if self.training_dataloader is None:
            self.tput_timer.start()
        # slots of the layer-stacked activation buffers taken by this forward stay its own until a
        # backward runs through its graph (ops/wgrad_batch.py)
        wtag = _wgrad_batch.begin_forward() if self._defer_wgrad else None
        try:
            if self.amp is not None:
                with self.amp.autocast():
                    loss = self.module(*inputs, **kwargs)
            else:
                loss = self.module(*inputs, **kwargs)
        except BaseException:
            if wtag is not None:
                _wgrad_batch.end_forward(wtag, None)
            raise
        if wtag is not None:
            _wgrad_batch.end_forward(wtag, loss)
        if self.wall_clock_breakdown():
            self.timers("forward").stop()
            self.timers("forward_microstep").stop()
        if self.flops_profiler is not None and self.global_steps == self.flops_profiler_profile_step() and \
                self.global_rank == 0:
            self.flops_profiler.print_model_profile(profile_step=self.global_steps,
                                                    module_depth=self.flops_profiler_module_depth(),
                                                    top_modules=self.flops_profiler_top_modules(),
                                                    detailed=self.flops_profiler_detailed())
            self.flops_profiler.end_profile()
            self.flops_profiler = None
        return loss

    def allreduce_gradients(self, bucket_size=MEMORY_OPT_ALLREDUCE_SIZE):
        if self.zero_optimization() or (self.fp16_enabled() and hasattr(self.optimizer, "reduce_epilogue")):
            if hasattr(self.optimizer, "reduce_epilogue"):
                self.optimizer.reduce_epilogue()
            return
        if self.is_gradient_accumulation_boundary() and dist.is_initialized() and self.dp_world_size > 1:
            self.buffered_allreduce_fallback(elements_per_buffer=bucket_size)

    def backward(self, loss, allreduce_gradients=True, release_loss=False):
        with comm.trace_range("engine.backward"):
            return self._backward_impl(loss, allreduce_gradients, release_loss)

    def _backward_impl(self, loss, allreduce_gradients=True, release_loss=False):
        if not allreduce_gradients:
            logger.warning("Argument `allreduce_gradients` is deprecated, ignored, and will soon be removed")
        if self.gradient_accumulation_steps() > 1:
            loss = self._scale_loss(loss.float())
        if self.tensorboard_enabled() and self.is_gradient_accumulation_boundary() and self.global_rank == 0:
            self.summary_writer.add_scalar("Train/Samples/train_loss",
                                           loss.mean().item() * self.gradient_accumulation_steps(),
                                           self.global_samples)
            self.summary_writer.flush()
        if self.wall_clock_breakdown():
            self.timers("backward_microstep").start()
            self.timers("backward").start()
        assert self.optimizer is not None, "must provide optimizer during init in order to use backward"
        if self.wall_clock_breakdown():
            self.timers("backward_inner_microstep").start()
            self.timers("backward_inner").start()
        if hasattr(self.optimizer, "is_gradient_accumulation_boundary"):
            self.optimizer.is_gradient_accumulation_boundary = self.is_gradient_accumulation_boundary()
        # weight gradients deferred to one batched GEMM per shape at the end of this backward,
        # where nothing reads gradients before it returns (ops/linear.py deferred_wgrads)
        with _wgrad_batch.deferred(self._defer_wgrad):
            if hasattr(self.optimizer, "backward") and (self.zero_optimization() or self.fp16_enabled()):
                self.optimizer.backward(loss)
            elif self.amp is not None:
                # the unscale is delayed to the accumulation boundary (apex delay_unscale)
                self.amp.scale(loss).backward()
            else:
                loss.backward()
        _linear_ops.end_backward_pass()  # pre-transposed operands never outlive their backward
        if self.wall_clock_breakdown():
            self.timers("backward_inner").stop()
            self.timers("backward_inner_microstep").stop()
            self.timers("backward_allreduce_microstep").start()
            self.timers("backward_allreduce").start()
        if self.enable_backward_allreduce:
            self.allreduce_gradients()
        if self.wall_clock_breakdown():
            self.timers("backward_allreduce").stop()
            self.timers("backward_allreduce_microstep").stop()
            self.timers("backward").stop()
            self.timers("backward_microstep").stop()
        return loss

    def is_gradient_accumulation_boundary(self):
        return (self.micro_steps + 1) % self.gradient_accumulation_steps() == 0

    def set_batch_shape(self, micro_batch: int, grad_accum: int):
        """Re-split the per-rank batch (micro_batch x grad_accum, same product) between two
        optimizer steps -- a trainer trading micro-batch activations for HBM.  Only legal at a
        step boundary; the train batch size is unchanged."""
        if self.micro_steps % self.gradient_accumulation_steps() != 0:
            raise RuntimeError("set_batch_shape() must be called at an optimizer-step boundary")
        c = self._config
        if micro_batch * grad_accum != c.train_micro_batch_size_per_gpu * c.gradient_accumulation_steps:
            raise ValueError("set_batch_shape() keeps train_batch_size: micro_batch * grad_accum must not change")
        c.train_micro_batch_size_per_gpu = int(micro_batch)
        c.gradient_accumulation_steps = int(grad_accum)
        self.micro_steps = 0
        opt = self.optimizer
        if hasattr(opt, "gradient_accumulation_steps"):
            opt.gradient_accumulation_steps = int(grad_accum)
            if hasattr(opt, "refresh_grad_dtype"):  # the reduced-gradient dtype depends on GA
                opt.refresh_grad_dtype()

    def zero_grad(self):
        if hasattr(self.optimizer, "groups"):
            self.optimizer.zero_grad()
            return
        for _, param in self.module.named_parameters():
            param.grad = None

    def clip_fp32_gradients(self):
        clip_grad_norm_(parameters=self.module.parameters(), max_norm=self.gradient_clipping(), mpu=self.mpu)

    def _snapshot_gradients(self):
        if hasattr(self.optimizer, "groups"):  # flat-arena optimizers: per-param views of reduced grads
            grads = []
            for p in self.module.parameters():
                g = p.grad if p.grad is not None else torch.zeros_like(p)
                grads.append(g.detach().clone().cpu() if self.store_gradients_cpu else g.detach().clone())
            return grads
        return [(p.grad.clone().cpu() if self.store_gradients_cpu else p.grad.clone()) if p.grad is not None else None
                for p in self.module.parameters()]

    def _take_model_step(self, lr_kwargs):
        if self.gradient_clipping() > 0.0 and not self.fp16_enabled() and not hasattr(self.optimizer, "groups"):
            self.timers("_step_clipping").start()
            if self.amp is not None:
                self.amp.unscale(self.optimizer)  # clip the unscaled fp32 masters (REF engine.py:1148-1153)
            self.clip_fp32_gradients()
            self.timers("_step_clipping").stop()
        if self.store_gradients:
            if self.amp is not None:
                self.amp.unscale(self.optimizer)
            self.stored_gradients = self._snapshot_gradients()
        self.timers("_step_step").start()
        if self.amp is not None:
            self.amp.step(self.optimizer)
        else:
            self.optimizer.step()
        self.timers("_step_step").stop()
        self.timers("_step_zero_grad").start()
        if hasattr(self.optimizer, "groups"):
            pass  # flat-arena optimizers zero their own gradient storage inside step()
        elif not self.zero_optimization() and not self.fp16_enabled() and not self.amp_enabled():
            self.zero_grad()
        else:
            self.optimizer.zero_grad()
        self.timers("_step_zero_grad").stop()
        report_progress = self.global_rank == 0
        overflow = bool(self.amp.overflow if self.amp is not None else getattr(self.optimizer, "overflow", False))
        if overflow:
            self.skipped_steps += 1
        elif self.lr_scheduler is not None:
            self.lr_scheduler.step(**(lr_kwargs or {}))
        if (self.global_steps + 1) % self.steps_per_print() == 0:
            # every rank reconciles at the same boundary: the roll-back of the optimizer's step
            # counters must stay identical across data-parallel replicas
            self._reconcile_device_skips()
            if report_progress:
                self._report_progress(self.global_steps + 1)
        self.global_steps += 1
        self.global_samples += self.train_batch_size()

    def step(self, lr_kwargs=None):
        with comm.trace_range("engine.step"):
            return self._step_impl(lr_kwargs)

    def _step_impl(self, lr_kwargs=None):
        if self.wall_clock_breakdown():
            self.timers("step_microstep").start()
            self.timers("step").start()
        assert self.optimizer is not None, "must provide optimizer during init in order to use step"
        report_progress = self.global_rank == 0
        if self.is_gradient_accumulation_boundary():
            if self.progressive_layer_drop:
                self.progressive_layer_drop.update_state(self.global_steps)
            self._take_model_step(lr_kwargs)
        self.tput_timer.stop(report_progress)
        if self.tensorboard_enabled() and self.is_gradient_accumulation_boundary() and self.global_rank == 0:
            self.summary_writer.add_scalar("Train/Samples/lr", self.get_lr()[0], self.global_samples)
            if self.fp16_enabled() and hasattr(self.optimizer, "cur_scale"):
                self.summary_writer.add_scalar("Train/Samples/loss_scale", self.optimizer.cur_scale,
                                               self.global_samples)
            self.summary_writer.flush()
        if self.wall_clock_breakdown():
            self.timers("step").stop()
            self.timers("step_microstep").stop()
            self.timers.log(names=["forward_microstep", "backward_microstep", "backward_inner_microstep",
                                   "backward_allreduce_microstep", "step_microstep"],
                            memory_breakdown=self.memory_breakdown())
            if self.is_gradient_accumulation_boundary():
                self.timers.log(["forward", "backward", "backward_inner", "backward_allreduce", "step"])
        self.micro_steps += 1

    def _get_optimizer_param(self, param_name):
        if not self.optimizer:
            return []
        return [g.get(param_name, 0.0) for g in self.optimizer.param_groups]

    def get_lr(self):
        return self._get_optimizer_param("lr")

    def get_type(self):
        return self._get_optimizer_param("type")

    def get_mom(self):
        if self.optimizer_name() in ["SGD", "RMSprop"]:
            return self._get_optimizer_param("momentum")
        return self._get_optimizer_param("betas")

    def get_pld_theta(self):
        return self.progressive_layer_drop.get_theta() if self.progressive_layer_drop else None

    def _reconcile_device_skips(self):
        """Steps the optimizer skipped on the device without a host sync (sync-free LAMB)."""
        if hasattr(self.optimizer, "reconcile_skipped_steps"):
            self.skipped_steps += self.optimizer.reconcile_skipped_steps()

    def _report_progress(self, step):
        log_dist(f"step={step}, skipped={self.skipped_steps}, lr={self.get_lr()}, mom={self.get_mom()}", ranks=[0])

    # ------------------------------------------------------------------ fp32 / client-optimizer all-reduce
    def allreduce_bucket(self, bucket):
        tensor = self.flatten(bucket)
        t = tensor.float() if self.allreduce_always_fp32() else tensor
        if self.postscale_gradients():
            if self.gradient_predivide_factor() != 1.0:
                t.mul_(1.0 / self.gradient_predivide_factor())
            dist.all_reduce(t, group=self.data_parallel_group)
            if self.gradient_average and self.gradient_predivide_factor() != self.dp_world_size:
                t.mul_(self.gradient_predivide_factor() / self.dp_world_size)
        else:
            t.div_(self.dp_world_size)
            dist.all_reduce(t, group=self.data_parallel_group)
        if self.allreduce_always_fp32() and tensor is not t:
            tensor.copy_(t)
        return tensor

    def allreduce_and_copy(self, small_bucket):
        allreduced = self.allreduce_bucket(small_bucket)
        for buf, synced in zip(small_bucket, self.unflatten(allreduced, small_bucket)):
            buf.copy_(synced)

    def allreduce_no_retain(self, bucket, numel_per_bucket=500000000):
        small, numel = [], 0
        for t in bucket:
            small.append(t)
            numel += t.numel()
            if numel > numel_per_bucket:
                self.allreduce_and_copy(small)
                small, numel = [], 0
        if small:
            self.allreduce_and_copy(small)

    def buffered_allreduce_fallback(self, grads=None, elements_per_buffer=500000000):
        grads = []
        for name, p in self.module.named_parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            g = p.grad
            if g.is_sparse and self.sparse_gradients_enabled():
                grads.append(("csr", name, p))
            else:
                grads.append(("dense", name, g.data))
        dense = [g for kind, _, g in grads if kind == "dense"]
        for bucket in split_half_float_double_csr(dense):
            self.allreduce_no_retain(bucket, numel_per_bucket=elements_per_buffer)
        for kind, _, p in grads:
            if kind == "csr":
                from .csr_tensor import CSRTensor
                csr = CSRTensor(p.grad)
                self.csr_allreduce(csr)
                p.grad = csr.to_dense()

    def csr_allreduce(self, csr):
        csr.values.div_(self.dp_world_size)
        idx_list = self.csr_all_gather(csr.indices)
        val_list = self.csr_all_gather(csr.values)
        csr.indices = torch.cat(idx_list)
        csr.values = torch.cat(val_list)
        return csr

    def csr_all_gather(self, value):
        my_size = torch.LongTensor([value.size()[0]]).to(value.device)
        all_sizes = [torch.zeros_like(my_size) for _ in range(self.dp_world_size)]
        dist.all_gather(all_sizes, my_size, group=self.data_parallel_group)
        max_size = int(torch.cat(all_sizes).max())
        fill = max_size - int(my_size)
        if value.dim() == 1:
            padded = torch.cat([value, value.new_zeros(fill)]) if fill > 0 else value
        else:
            padded = torch.cat([value, value.new_zeros(fill, value.size(1))]) if fill > 0 else value
        tensor_list = [torch.zeros_like(padded) for _ in range(self.dp_world_size)]
        dist.all_gather(tensor_list, padded, group=self.data_parallel_group)
        return [t[: int(s)] for t, s in zip(tensor_list, all_sizes)]

    # ------------------------------------------------------------------ checkpointing
    def _get_ckpt_name(self, checkpoints_path, tag, mp_placeholder=None):
        mp_rank = self.mpu.get_model_parallel_rank() if self.mpu is not None else 0
        mp_rank_str = mp_placeholder if mp_placeholder is not None else f"{mp_rank:02d}"
        if self.zero_optimization_partition_weights():
            dp = dist.get_rank(group=self.optimizer.dp_group) if dist.is_initialized() else 0
            filename = "zero_pp_rank_{}".format(dp)
            return os.path.join(checkpoints_path, str(tag), f"{filename}_mp_rank_{mp_rank_str}_model_states.pt")
        return os.path.join(checkpoints_path, str(tag), f"mp_rank_{mp_rank_str}_model_states.pt")

    def _get_zero_ckpt_name(self, checkpoints_path, tag, dp_rank=None):
        mp_rank = self.mpu.get_model_parallel_rank() if self.mpu is not None else 0
        pp = dist.get_rank(group=self.optimizer.dp_group) if (dp_rank is None and dist.is_initialized()) else \
            (dp_rank or 0)
        return os.path.join(checkpoints_path, str(tag), f"zero_pp_rank_{pp}_mp_rank_{mp_rank:02d}_optim_states.pt")

    def _get_all_zero_checkpoint_names(self, load_dir, tag, mp_world_size, dp_world_size):
        mp_rank = self.mpu.get_model_parallel_rank() if self.mpu is not None else 0
        return [os.path.join(load_dir, str(tag), f"zero_pp_rank_{dp}_mp_rank_{mp_rank:02d}_optim_states.pt")
                for dp in range(dp_world_size)]

    def _checkpoint_tag_validation(self, tag):
        if not self._config.checkpoint_tag_validation_enabled or not dist.is_initialized():
            return
        s_hash = hashlib.sha1(str(tag).encode())
        bhash = torch.ByteTensor([s_hash.digest()]).flatten().to(self.device)
        max_bhash, min_bhash = bhash.clone(), bhash.clone()
        dist.all_reduce(max_bhash, op=dist.ReduceOp.MAX)
        dist.all_reduce(min_bhash, op=dist.ReduceOp.MIN)
        valid = torch.all(min_bhash == bhash) and torch.all(max_bhash == bhash)
        msg = f"[rank={dist.get_rank()}] The checkpoint tag name '{tag}' is not consistent across all ranks. " \
              "Including rank unique information in checkpoint tag could cause issues when restoring with " \
              "different world sizes."
        if self._config.checkpoint_tag_validation_fail:
            assert valid, msg
        elif not valid:
            logger.warning(msg)

    def synchronize(self):
        """Order the current stream after an overlapped optimizer step (zero_optimization.overlap_step)."""
        sync = getattr(self.optimizer, "synchronize_step", None)
        if sync is not None:
            sync()

    def module_state_dict(self, destination=None, prefix="", keep_vars=False):
        self.synchronize()
        return self.module.state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)

    def load_module_state_dict(self, state_dict, strict=True):
        self.module.load_state_dict(state_dict, strict=strict)

    def save_checkpoint(self, save_dir, tag=None, client_state=None, save_latest=True):
        self.synchronize()
        client_state = client_state or {}
        if self.zero_optimization_partition_weights():
            pass  # shards are always in partitioned form
        if tag is None:
            tag = f"global_step{self.global_steps}"
        tag = str(tag)
        self._checkpoint_tag_validation(tag)
        self._reconcile_device_skips()  # on every rank, not only the ones that write the model file
        if self.save_non_zero_checkpoint:
            self._create_checkpoint_file(save_dir, tag, False)
            self._save_checkpoint(save_dir, tag, client_state=client_state)
        if self.save_zero_checkpoint:
            self._create_zero_checkpoint_files(save_dir, tag)
            self._save_zero_checkpoint(save_dir, tag)
        if dist.is_initialized():
            dist.barrier()
        if save_latest and self.global_rank == 0:
            with open(os.path.join(save_dir, "latest"), "w") as fd:
                fd.write(tag)
        if dist.is_initialized():
            dist.barrier()
        return True

    def _create_checkpoint_file(self, save_dir, tag, zero_checkpoint):
        name_function = self._get_zero_ckpt_name if zero_checkpoint else self._get_ckpt_name
        checkpoint_name = name_function(save_dir, tag)
        os.makedirs(os.path.dirname(checkpoint_name), exist_ok=True)

    def _create_zero_checkpoint_files(self, save_dir, tag):
        self._create_checkpoint_file(save_dir, tag, True)

    def _zero3_module_payload(self):
        opt = self.optimizer
        from .zero.layout import layout_signature
        return {"zero3_param_shards": [opt.param_shard_host(g) for g in opt.groups],
                "layout": layout_signature(opt.groups), "dp_world_size": opt.dp_world}

    def _save_checkpoint(self, save_dir, tag, client_state=None):
        self._reconcile_device_skips()
        save_path = self._get_ckpt_name(save_dir, tag)
        if self.zero_optimization_partition_weights():
            module_sd = self._zero3_module_payload()
        else:
            module_sd = self.module_state_dict()
        state = dict(module=module_sd,
                     optimizer=self.optimizer.state_dict() if self.optimizer and not self.zero_optimization() else None,
                     lr_scheduler=self.lr_scheduler.state_dict() if self.lr_scheduler is not None else None,
                     csr_tensor_module_names=self.csr_tensor_module_names, skipped_steps=self.skipped_steps,
                     global_steps=self.global_steps, global_samples=self.global_samples,
                     dp_world_size=self.dp_world_size, mp_world_size=self.mp_world_size, ds_version=__version__)
        if self.amp is not None:
            state["amp"] = self.amp.state_dict()
        state.update(client_state or {})
        log_dist(message=f"Saving model checkpoint: {save_path}", ranks=[0])
        torch.save(state, save_path)

    def _copy_recovery_script(self, save_path):
        base_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        script = "zero_to_fp32.py"
        src = os.path.join(base_dir, "utils", script)
        dst = os.path.join(save_path, script)
        if os.path.exists(src):
            shutil.copyfile(src, dst)

    def _save_zero_checkpoint(self, save_path, tag):
        zero_checkpoint_name = self._get_zero_ckpt_name(save_path, tag)
        if getattr(self._config, "checkpoint_zero_format", "native") == "reference":
            zero_sd = self._reference_zero_state()
        else:
            zero_sd = dict(optimizer_state_dict=self.optimizer.state_dict(),
                           param_shapes=self._get_zero_param_shapes(), ds_version=__version__)
        torch.save(zero_sd, zero_checkpoint_name)
        self._copy_recovery_script(os.path.dirname(zero_checkpoint_name))
        log_dist(f"zero checkpoint saved {zero_checkpoint_name}", ranks=[0])

    def _reference_zero_state(self):
        """ZeRO optimizer file in the reference layout (checkpoint.zero_format = "reference"):
        contiguous per-group fp32 partitions under the reference's keys, `param_shapes` as the
        reference writes it (every module parameter in order, reference engine.py:1792-1798),
        plus each optimizer group's parameter names so multi-group files consolidate exactly."""
        from .zero.ref_layout import export_reference_state_dict
        opt = self.optimizer
        self.synchronize()
        osd = export_reference_state_dict(opt, max_elems_per_comm=int(self.zero_reduce_bucket_size()),
                                          sub_group_size=int(self.zero_sub_group_size()))
        names = {id(p): n for n, p in self.module.named_parameters()}
        shapes = OrderedDict((n, torch.Size(getattr(p, "ds_shape", p.shape))) for n, p in self.module.named_parameters())
        groups = [[names.get(id(p), str(id(p))) for p in plist] for plist in opt._orig_group_params]
        return dict(optimizer_state_dict=osd, param_shapes=shapes, dsa_group_param_names=groups,
                    ds_version=__version__)

    def _get_zero_param_shapes(self):
        names = {id(p): n for n, p in self.module.named_parameters()}
        out = []
        for g in self.optimizer.groups:
            d = OrderedDict()
            for p in g.params:
                d[names.get(id(p), str(id(p)))] = tuple(getattr(p, "ds_shape", p.shape))
            out.append(d)
        return out

    @staticmethod
    def _load_file(path, map_location="cpu"):
        """Weights-only load.  Types this framework itself writes into checkpoints, plus
        argparse.Namespace (GPT-NeoX client state), are allow-listed; anything else in the
        file is refused unless DSA_ALLOW_UNSAFE_CHECKPOINT_LOAD=1 explicitly opts into full
        unpickling of a trusted file."""
        import argparse
        import pickle
        from .fp16.loss_scaler import DynamicLossScaler, LossScaler
        # reference checkpoints pickle their loss-scaler object: the same attribute set as
        # ours, reconstructed without running any code from the file
        safe = [argparse.Namespace, set, OrderedDict,
                (DynamicLossScaler, "deepspeed.runtime.fp16.loss_scaler.DynamicLossScaler"),
                (LossScaler, "deepspeed.runtime.fp16.loss_scaler.LossScaler")]
        try:
            with torch.serialization.safe_globals(safe):
                return torch.load(path, map_location=map_location, weights_only=True)
        except pickle.UnpicklingError as e:
            if os.environ.get("DSA_ALLOW_UNSAFE_CHECKPOINT_LOAD", "0") == "1":
                logger.warning(f"{path}: not loadable weights-only ({e}); DSA_ALLOW_UNSAFE_CHECKPOINT_LOAD=1 set, "
                               f"unpickling the full file")
                return torch.load(path, map_location=map_location, weights_only=False)
            raise RuntimeError(f"{path} holds objects outside the weights-only allow-list: {e}. Register the "
                               f"types with torch.serialization.add_safe_globals, or set "
                               f"DSA_ALLOW_UNSAFE_CHECKPOINT_LOAD=1 for a file you trust.") from e

    def load_checkpoint(self, load_dir, tag=None, load_module_strict=True, load_optimizer_states=True,
                        load_lr_scheduler_states=True):
        self.synchronize()
        if tag is None:
            latest_path = os.path.join(load_dir, "latest")
            if os.path.isfile(latest_path):
                with open(latest_path, "r") as fd:
                    tag = fd.read().strip()
            else:
                logger.warning(f"Unable to find latest file at {latest_path}, if trying to load latest checkpoint "
                               "please ensure this file exists or pass an explicit checkpoint tag when loading a "
                               "checkpoint.")
                return None, None
        load_path, client_states = self._load_checkpoint(load_dir, tag, load_module_strict=load_module_strict,
                                                         load_optimizer_states=load_optimizer_states,
                                                         load_lr_scheduler_states=load_lr_scheduler_states)
        if self.zero_optimization() and load_path is not None:
            self._load_zero_checkpoint(load_dir, tag, load_optimizer_states=load_optimizer_states)
        return load_path, client_states

    def _load_checkpoint(self, load_dir, tag, load_module_strict=True, load_optimizer_states=True,
                         load_lr_scheduler_states=True):
        load_path = self._get_ckpt_name(load_dir, tag)
        if not os.path.exists(load_path) and self.zero_optimization_partition_weights():
            # ZeRO-3 model states are written per data-parallel rank: a larger world than the
            # saving one reads rank 0's (its parameter shards are re-partitioned from every
            # saved rank's file, _load_zero3_module)
            alt = os.path.join(os.path.dirname(load_path),
                               "zero_pp_rank_0_mp_rank_" + os.path.basename(load_path).split("_mp_rank_")[1])
            if os.path.exists(alt):
                load_path = alt
        if not os.path.exists(load_path):
            logger.warning("Client provided checkpoint load path: {} does not exist ... skip checkpoint load"
                           .format(load_path))
            return None, None
        logger.info(f"rank: {self.global_rank} loading checkpoint: {load_path}")
        checkpoint = self._load_file(load_path)
        if self.zero_optimization_partition_weights():
            self._load_zero3_module(checkpoint["module"], load_path)
        elif checkpoint.get("module") is not None or getattr(self, "_loads_module_from_dir", False):
            self.load_module_state_dict(state_dict=checkpoint.get("module"), strict=load_module_strict)
            if hasattr(self.optimizer, "refresh_from_params") and (not load_optimizer_states or
                                                                  not self.zero_optimization()):
                self.optimizer.refresh_from_params()
        if not self.zero_optimization() and load_optimizer_states and self.optimizer is not None and \
                checkpoint.get("optimizer") is not None:
            self.optimizer.load_state_dict(checkpoint["optimizer"])
        if self.amp is not None and load_optimizer_states and checkpoint.get("amp"):
            self.amp.load_state_dict(checkpoint["amp"])
        if load_lr_scheduler_states and self.lr_scheduler is not None and checkpoint.get("lr_scheduler"):
            self.lr_scheduler.load_state_dict(checkpoint["lr_scheduler"])
        self.csr_tensor_module_names = checkpoint.get("csr_tensor_module_names", set())
        self.global_steps = checkpoint.get("global_steps", 0)
        self.global_samples = checkpoint.get("global_samples", self.global_steps * self.train_batch_size())
        self.skipped_steps = checkpoint.get("skipped_steps", 0)
        self.loaded_checkpoint_mp_world_size = checkpoint.get("mp_world_size")
        self.loaded_checkpoint_dp_world_size = checkpoint.get("dp_world_size")
        deepspeed_states = ["module", "optimizer", "amp", "lr_scheduler", "csr_tensor_module_names", "skipped_steps",
                            "global_steps", "dp_world_size", "mp_world_size", "global_samples", "ds_version"]
        client_state = {k: v for k, v in checkpoint.items() if k not in deepspeed_states}
        return load_path, client_state

    def _load_zero3_module(self, payload, load_path=None):
        """Restore this rank's ZeRO-3 bf16 parameter shards.  Same layout and DP world: the
        saved shard as is.  Otherwise the low-precision parameters are rebuilt from every
        saved rank's shard (zero_pp_rank_*_model_states.pt) and re-partitioned, so that a
        load with load_from_fp32_weights=false still restores the weights."""
        opt = self.optimizer
        if payload is None or "zero3_param_shards" not in payload:
            return
        from .zero.layout import layout_signature, params_to_shard, shards_to_params
        if payload.get("layout") == layout_signature(opt.groups) and payload.get("dp_world_size") == opt.dp_world:
            for g, s in zip(opt.groups, payload["zero3_param_shards"]):
                opt.load_param_shard(g, s)
            opt._post_step()
            return
        old_world = int(payload.get("dp_world_size") or 1)
        folder = os.path.dirname(load_path) if load_path else None
        mp = os.path.basename(load_path).split("_mp_rank_")[1] if load_path else "00_model_states.pt"
        files = [os.path.join(folder, f"zero_pp_rank_{r}_mp_rank_{mp}") for r in range(old_world)] if folder else []
        if not files or not all(os.path.exists(f) for f in files):
            logger.warning("ZeRO-3 checkpoint: layout / DP world changed and not every rank's model-states file is "
                           "present; parameters are restored from the fp32 masters only")
            return
        payloads = [self._load_file(f)["module"] for f in files]
        sigs = payloads[0]["layout"]
        for gi, g in enumerate(opt.groups):
            full = shards_to_params([pl["zero3_param_shards"][gi] for pl in payloads], sigs[gi])
            opt.load_param_shard(g, params_to_shard(full, g, opt.dp_rank, g.dtype))
        logger.info(f"ZeRO-3 checkpoint: re-partitioned bf16 parameters from {old_world} to {opt.dp_world} ranks")
        opt._post_step()

    def _load_zero_checkpoint(self, load_dir, tag, load_optimizer_states=True):
        dp_world = self.loaded_checkpoint_dp_world_size or self.dp_world_size
        names = self._get_all_zero_checkpoint_names(load_dir, tag, self.mp_world_size, dp_world)
        names = [n for n in names if os.path.exists(n)]
        if not names:
            logger.warning(f"No ZeRO optimizer checkpoint found under {load_dir}/{tag}")
            return
        sds = [self._load_file(n)["optimizer_state_dict"] for n in names]
        self.optimizer.load_state_dict(state_dict_list=sds, load_optimizer_states=load_optimizer_states,
                                       load_from_fp32_weights=self.zero_load_from_fp32_weights())
        log_dist(f"loading {len(sds)} zero partition checkpoints for rank {self.global_rank}", ranks=[0])

    def _zero3_consolidated_fp16_state_dict(self):
        return self.optimizer.gathered_state_dict(self.module)

    def save_fp16_model(self, save_dir, save_filename="pytorch_model.bin"):
        path = os.path.join(save_dir, save_filename)
        if self.zero_optimization_partition_weights():
            if not self.zero_gather_fp16_weights_on_model_save():
                logger.warning("stage3_gather_fp16_weights_on_model_save=false. save_fp16_model saved nothing.")
                return
            sd = self._zero3_consolidated_fp16_state_dict()
        else:
            sd = self.module_state_dict()
        if self.global_rank == 0:
            os.makedirs(save_dir, exist_ok=True)
            logger.info(f"Saving model weights to {path}")
            torch.save(sd, path)


class _NullSummaryWriter:
    """Fallback when tensorboard is unavailable: writes scalars as text lines."""

    def __init__(self, log_dir):
        self.path = os.path.join(log_dir, "scalars.tsv")

    def add_scalar(self, tag, value, step):
        with open(self.path, "a") as f:
            f.write(f"{tag}\t{step}\t{value}\n")

    def flush(self):
        pass
