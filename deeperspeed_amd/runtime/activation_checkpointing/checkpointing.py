"""Activation checkpointing (Megatron-compatible API).

Reference parity: deepspeed/runtime/activation_checkpointing/checkpointing.py:1-861 --
`checkpoint(function, *args)` with recompute in backward, RNG state replay (host + device
+ model-parallel tracker), `partition_activations` (each model-parallel rank keeps 1/mp of
every checkpointed activation and all-gathers before recompute), `contiguous_memory_optimization`
(checkpoint shards live in one pre-sized buffer), `cpu_checkpointing` (shards parked in
pinned host memory), `synchronize_checkpoint_boundary`, `profile` timers, and
`configure(...)` / `is_configured()` / `reset()` / `model_parallel_cuda_manual_seed`.

Implementation notes (MI355X): shard transfers to/from host use non-blocking copies from
pinned buffers; the partition all-gather is one `all_gather_into_tensor`.
"""

from __future__ import annotations

import contextlib
import copy

import torch
import torch.distributed as dist

from ...utils.logging import logger
from ...utils.timer import SynchronizedWallClockTimer

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"

mpu = None
num_layers = None
PARTITION_ACTIVATIONS = False
CONTIGUOUS_CHECKPOINTING = False
CPU_CHECKPOINT = False
SYNCHRONIZE = False
PROFILE_TIME = False
deepspeed_checkpointing_enabled = False
timers = None
_contiguous_buffers = []
_contiguous_index = 0


def _set_cuda_rng_state(new_state, device=-1):
    if not torch.cuda.is_available():
        return
    torch.cuda.set_rng_state(new_state)


class CudaRNGStatesTracker:
    """Tracks named device RNG states (model-parallel regions use a different stream of
    random numbers per rank for dropout while the default state stays identical)."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return copy.copy(self.states_)

    def set_states(self, states):
        self.states_ = states

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception("seed {} already exists".format(seed))
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception("cuda rng state {} already exists".format(name))
        if not torch.cuda.is_available():
            g = torch.Generator()
            g.manual_seed(seed)
            self.states_[name] = g.get_state()
            return
        orig = torch.cuda.get_rng_state()
        torch.cuda.manual_seed(seed)
        self.states_[name] = torch.cuda.get_rng_state()
        _set_cuda_rng_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception("cuda rng state {} is not added".format(name))
        if not torch.cuda.is_available():
            yield
            return
        orig = torch.cuda.get_rng_state()
        _set_cuda_rng_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = torch.cuda.get_rng_state()
            _set_cuda_rng_state(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    """Default state: `seed`; tensor-model-parallel state: seed + 2718 + mp_rank."""
    tp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
    offset = seed + 2718
    model_parallel_seed = offset + tp_rank
    data_parallel_seed = seed
    if dist.is_initialized() and dist.get_rank() == 0:
        logger.info("> initializing model parallel cuda seeds on global rank {}, model parallel rank {}, and data "
                    "parallel rank {} with model parallel seed: {} and data parallel seed: {}".format(
                        dist.get_rank(), tp_rank, mpu.get_data_parallel_rank() if mpu else 0, model_parallel_seed,
                        data_parallel_seed))
    _CUDA_RNG_STATE_TRACKER.reset()
    if torch.cuda.is_available():
        torch.cuda.manual_seed(data_parallel_seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, model_parallel_seed)


def _mp_group_info():
    if mpu is None:
        return None, 1, 0
    return mpu.get_model_parallel_group(), mpu.get_model_parallel_world_size(), mpu.get_model_parallel_rank()


def _partition(t: torch.Tensor):
    """Keep this rank's 1/mp slice of a flat activation (padded)."""
    group, mp, rank = _mp_group_info()
    flat = t.detach().contiguous().view(-1)
    n = flat.numel()
    per = (n + mp - 1) // mp
    if per * mp != n:
        flat = torch.cat([flat, flat.new_zeros(per * mp - n)])
    part = flat[rank * per:(rank + 1) * per].clone()
    if CPU_CHECKPOINT:
        host = torch.empty(part.shape, dtype=part.dtype, pin_memory=torch.cuda.is_available())
        host.copy_(part, non_blocking=True)
        part = host
    elif CONTIGUOUS_CHECKPOINTING:
        part = _contiguous_store(part)
    return (part, tuple(t.shape), n, t.device)


def _contiguous_store(part):
    global _contiguous_index
    need = part.numel()
    for buf in _contiguous_buffers:
        if buf["dtype"] == part.dtype and buf["used"] + need <= buf["tensor"].numel():
            view = buf["tensor"][buf["used"]: buf["used"] + need]
            buf["used"] += need
            view.copy_(part)
            return view
    size = max(need * (num_layers or 1), need)
    t = torch.empty(size, dtype=part.dtype, device=part.device)
    _contiguous_buffers.append({"tensor": t, "used": need, "dtype": part.dtype})
    t[:need].copy_(part)
    return t[:need]


def _gather(rec):
    part, shape, n, device = rec
    group, mp, rank = _mp_group_info()
    part = part.to(device, non_blocking=True)
    if mp == 1:
        return part[:n].view(shape)
    full = torch.empty(part.numel() * mp, dtype=part.dtype, device=device)
    dist.all_gather_into_tensor(full, part.contiguous(), group=group)
    return full[:n].view(shape)


_RECOMPUTE_DEPTH = 0
_CKPT_FWD_DEPTH = 0


def is_recomputing() -> bool:
    """True while a checkpointed function is being re-run inside backward.  Modules whose
    forward OUTPUT is not needed by any backward (e.g. the projection that feeds only a residual
    sum) can skip computing it then and produce gradients only (models/gpt_neox.py
    OutputLinear)."""
    return _RECOMPUTE_DEPTH > 0


def is_checkpoint_forward() -> bool:
    """True during the first (no_grad) forward of a checkpointed function: values computed now
    are discarded and recomputed in backward unless a module keeps them (selective recompute,
    models/gpt_neox.py NeoXAttention.stash_outputs)."""
    return _CKPT_FWD_DEPTH > 0


class CheckpointFunction(torch.autograd.Function):
    """Reentrant checkpoint: forward under no_grad, recompute inside backward."""

    @staticmethod
    def forward(ctx, run_function, *args):
        ctx.run_function = run_function
        if timers is not None and PROFILE_TIME:
            timers("forward").start()
        ctx.fwd_cpu_rng_state = torch.get_rng_state()
        ctx.fwd_cuda_rng_state = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        ctx.fwd_cuda_rng_state_tracker = get_cuda_rng_tracker().get_states()
        global _CKPT_FWD_DEPTH
        _CKPT_FWD_DEPTH += 1
        try:
            with torch.no_grad():
                outputs = run_function(*args)
        finally:
            _CKPT_FWD_DEPTH -= 1
        tensor_idx, saved, non_tensors = [], [], []
        for i, a in enumerate(args):
            if torch.is_tensor(a):
                if PARTITION_ACTIVATIONS and i == 0 and a.is_floating_point():
                    ctx.partitioned = _partition(a)
                    saved.append(None)
                    ctx.req_grad0 = a.requires_grad
                else:
                    saved.append(a)
                tensor_idx.append(i)
            else:
                non_tensors.append((i, a))
        if not PARTITION_ACTIVATIONS or not args or not torch.is_tensor(args[0]):
            ctx.partitioned = None
        ctx.tensor_idx = tensor_idx
        ctx.non_tensors = non_tensors
        ctx.nargs = len(args)
        ctx.save_for_backward(*[s for s in saved if s is not None])
        ctx.saved_mask = [s is not None for s in saved]
        if SYNCHRONIZE and torch.cuda.is_available():
            torch.cuda.synchronize()
        if timers is not None and PROFILE_TIME:
            timers("forward").stop()
        if torch.is_tensor(outputs):
            return outputs
        return tuple(outputs)

    @staticmethod
    def backward(ctx, *grads):
        if not torch.autograd._is_checkpoint_valid():
            raise RuntimeError("Checkpointing is not compatible with .grad(), please use .backward() if possible")
        if timers is not None and PROFILE_TIME:
            timers("backward").start()
        stored = list(ctx.saved_tensors)
        args = [None] * ctx.nargs
        k = 0
        for idx, has in zip(ctx.tensor_idx, ctx.saved_mask):
            if has:
                args[idx] = stored[k]
                k += 1
            else:
                full = _gather(ctx.partitioned)
                full.requires_grad_(ctx.req_grad0)
                args[idx] = full
        for i, a in ctx.non_tensors:
            args[i] = a
        detached = []
        for a in args:
            if torch.is_tensor(a):
                d = a.detach()
                d.requires_grad_(a.requires_grad)
                detached.append(d)
            else:
                detached.append(a)
        bwd_cpu_rng = torch.get_rng_state()
        bwd_cuda_rng = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        bwd_tracker = get_cuda_rng_tracker().get_states()
        torch.set_rng_state(ctx.fwd_cpu_rng_state)
        if ctx.fwd_cuda_rng_state is not None:
            _set_cuda_rng_state(ctx.fwd_cuda_rng_state)
        get_cuda_rng_tracker().set_states(ctx.fwd_cuda_rng_state_tracker)
        global _RECOMPUTE_DEPTH
        _RECOMPUTE_DEPTH += 1
        try:
            with torch.enable_grad():
                outputs = ctx.run_function(*detached)
        finally:
            _RECOMPUTE_DEPTH -= 1
        torch.set_rng_state(bwd_cpu_rng)
        if bwd_cuda_rng is not None:
            _set_cuda_rng_state(bwd_cuda_rng)
        get_cuda_rng_tracker().set_states(bwd_tracker)
        if torch.is_tensor(outputs):
            outputs = (outputs,)
        outs, gs = [], []
        for o, g in zip(outputs, grads):
            if torch.is_tensor(o) and o.requires_grad:
                outs.append(o)
                gs.append(g)
        if outs:
            torch.autograd.backward(outs, gs)
        if timers is not None and PROFILE_TIME:
            timers("backward").stop()
        return (None,) + tuple(d.grad if torch.is_tensor(d) else None for d in detached)


def checkpoint(function, *args):
    """Checkpoint a model or part of the model (returns function(*args))."""
    return CheckpointFunction.apply(function, *args)


def partition_activations_in_checkpoint(partition_activation):
    global PARTITION_ACTIVATIONS
    PARTITION_ACTIVATIONS = partition_activation
    if dist.is_initialized() and dist.get_rank() == 0:
        logger.info(f"**************Partition Activations {PARTITION_ACTIVATIONS}************")


def set_num_layers(nlayers):
    global num_layers
    num_layers = nlayers


def reset():
    """Reset contiguous buffers between iterations."""
    global _contiguous_index
    if CONTIGUOUS_CHECKPOINTING:
        for b in _contiguous_buffers:
            b["used"] = 0
    _contiguous_index = 0


def configure(mpu_, deepspeed_config=None, partition_activations=None, contiguous_checkpointing=None,
              num_checkpoints=None, checkpoint_in_cpu=None, synchronize=None, profile=None):
    global mpu, num_layers, deepspeed_checkpointing_enabled, PARTITION_ACTIVATIONS, CONTIGUOUS_CHECKPOINTING, \
        CPU_CHECKPOINT, SYNCHRONIZE, PROFILE_TIME, timers
    mpu = mpu_
    if deepspeed_config is not None:
        from ..config import DeepSpeedConfig
        cfg = deepspeed_config if isinstance(deepspeed_config, DeepSpeedConfig) else \
            DeepSpeedConfig(deepspeed_config, mpu=mpu_)
        ac = cfg.activation_checkpointing_config
        PARTITION_ACTIVATIONS = ac.partition_activations
        CONTIGUOUS_CHECKPOINTING = ac.contiguous_memory_optimization
        num_layers = ac.number_checkpoints
        CPU_CHECKPOINT = ac.cpu_checkpointing
        SYNCHRONIZE = ac.synchronize_checkpoint_boundary
        PROFILE_TIME = ac.profile
    if partition_activations is not None:
        PARTITION_ACTIVATIONS = partition_activations
    if contiguous_checkpointing is not None:
        CONTIGUOUS_CHECKPOINTING = contiguous_checkpointing
    if num_checkpoints is not None:
        num_layers = num_checkpoints
    if checkpoint_in_cpu is not None:
        CPU_CHECKPOINT = checkpoint_in_cpu
    if synchronize is not None:
        SYNCHRONIZE = synchronize
    if profile is not None:
        PROFILE_TIME = profile
    if CONTIGUOUS_CHECKPOINTING:
        assert PARTITION_ACTIVATIONS, "Contiguous Checkpointing is only availble with partitioned activations."
        assert num_layers is not None, "Must specify the number of layers with contiguous memory checkpointing"
    if PROFILE_TIME:
        timers = SynchronizedWallClockTimer()
    deepspeed_checkpointing_enabled = True


def is_configured():
    return deepspeed_checkpointing_enabled
