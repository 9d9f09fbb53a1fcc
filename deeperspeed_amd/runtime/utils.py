"""Runtime utilities (reference parity: deepspeed/runtime/utils.py).

Includes the layer partitioners used by the pipeline engine (`partition_uniform`,
`partition_balanced`), `PartitionedTensor` (activation sharding over a tensor-parallel
group), overflow / norm helpers, memory reporting and DeeperSpeed's
`GradientNoiseScale` (runtime/utils.py:618-674).
"""

import gc
import math
import os
import random
from bisect import bisect_left
from math import floor

import numpy as np
import torch
import torch.distributed as dist

from ..utils.logging import logger

try:
    import psutil
except ImportError:  # pragma: no cover
    psutil = None

torch_inf = float("inf")


def noop_decorator(func):
    return func


def ensure_directory_exists(filename):
    dirname = os.path.dirname(filename)
    os.makedirs(dirname, exist_ok=True)


def set_random_seed(seed):
    np.random.seed(seed)
    random.seed(seed)
    torch.manual_seed(seed)


def move_to_device(item, device):
    if torch.is_tensor(item):
        return item.to(device)
    if isinstance(item, list):
        return [move_to_device(v, device) for v in item]
    if isinstance(item, tuple):
        return tuple(move_to_device(v, device) for v in item)
    if isinstance(item, dict):
        return {k: move_to_device(v, device) for k, v in item.items()}
    return item


def is_model_parallel_parameter(p):
    return hasattr(p, "model_parallel") and p.model_parallel


def get_global_norm(norm_list):
    total = 0.0
    for n in norm_list:
        total += n ** 2.0
    return math.sqrt(total)


def call_to_str(base, *args, **kwargs):
    """Render `base(*args, **kwargs)` as a string (used for pipeline layer names)."""
    parts = [repr(a) for a in args] + [f"{k}={repr(v)}" for k, v in kwargs.items()]
    return f"{base}({', '.join(parts)})"


# ------------------------------------------------------------------------------ overflow / norms
class CheckOverflow:
    """Detect inf/nan in gradients across model- and data-parallel groups."""

    def __init__(self, param_groups=None, mpu=None, zero_reduce_scatter=False):
        self.mpu = mpu
        self.params = [] if param_groups else None
        self.zero_reduce_scatter = zero_reduce_scatter
        if param_groups:
            for group in param_groups:
                for p in group:
                    self.params.append(p)

    def check_using_norm(self, norm_group, reduce_overflow=True):
        overflow = -1 in norm_group
        if self.mpu is not None and dist.is_initialized():
            t = torch.tensor([1.0 if overflow else 0.0], device=_dev())
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.mpu.get_model_parallel_group())
            overflow = t.item() > 0
        elif reduce_overflow and dist.is_initialized():
            t = torch.tensor([1.0 if overflow else 0.0], device=_dev())
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            overflow = t.item() > 0
        return bool(overflow)

    def has_overflow_serial(self, params):
        for p in params:
            if p.grad is not None and self._has_inf_or_nan(p.grad.data):
                return True
        return False

    def has_overflow(self, params=None):
        params = self.params if params is None else params
        local = torch.zeros(1, device=_dev())
        for p in params:
            if p.grad is not None:
                local += (~torch.isfinite(p.grad.float())).any().float()
        if dist.is_initialized():
            dist.all_reduce(local, op=dist.ReduceOp.MAX)
            if self.mpu is not None:
                dist.all_reduce(local, op=dist.ReduceOp.MAX, group=self.mpu.get_model_parallel_group())
        return bool(local.item() > 0)

    @staticmethod
    def _has_inf_or_nan(x, j=None):
        s = float(x.float().sum())
        return s != s or s in (float("inf"), float("-inf"))


def _dev():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


_SUMSQ_MULTI = True  # False: torch _foreach_norm


def grad_norm_sq_tensor(parameters, mpu=None) -> torch.Tensor:
    """Sum of squared gradient entries as a 1-element fp32 tensor, without a host sync: one
    multi-tensor HIP reduction per (device, dtype) on the GPU (native.sumsq_multi_, fp32
    accumulation; torch's `_foreach_norm` elsewhere), model-parallel duplicates counted once,
    summed over the model-parallel group."""
    mp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
    grads = [p.grad.data for p in parameters if p.grad is not None and (mp_rank == 0 or is_model_parallel_parameter(p))]
    dev = grads[0].device if grads else _dev()
    acc = torch.zeros(1, device=dev, dtype=torch.float32)
    by_dev = {}
    for g in grads:
        by_dev.setdefault((g.device, g.dtype), []).append(g)
    for (d, dt), gs in by_dev.items():
        if (_SUMSQ_MULTI and d.type == "cuda" and d == acc.device
                and dt in (torch.float32, torch.bfloat16, torch.float16)):
            from ..ops import native
            native.sumsq_multi_([g.contiguous() for g in gs], acc)  # two HIP launches
        else:
            norms = torch._foreach_norm(gs, 2, dtype=torch.float32)
            acc += torch.stack(norms).square().sum().to(dev)
    if mpu is not None:
        dist.all_reduce(acc, group=mpu.get_model_parallel_group())
    return acc


def get_grad_norm(parameters, norm_type=2, mpu=None):
    """Global gradient norm; model-parallel duplicates counted once (on mp rank 0)."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = [p for p in parameters if p.grad is not None]
    norm_type = float(norm_type)
    mp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
    if norm_type == torch_inf:
        total = max([p.grad.data.abs().max().item() for p in parameters] + [0.0])
        t = torch.tensor([float(total)], device=_dev())
        if mpu is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=mpu.get_model_parallel_group())
        total = t.item()
    elif norm_type == 2.0:
        total = grad_norm_sq_tensor(parameters, mpu).item() ** 0.5
    else:
        acc = torch.zeros(1, device=_dev())
        for p in parameters:
            if mp_rank == 0 or is_model_parallel_parameter(p):
                acc += p.grad.data.float().norm(norm_type) ** norm_type
        if mpu is not None:
            dist.all_reduce(acc, group=mpu.get_model_parallel_group())
        total = acc.item() ** (1.0 / norm_type)
    if total in (float("inf"), -float("inf")) or total != total:
        total = -1
    return total


def get_weight_norm(parameters, norm_type=2, mpu=None):
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    norm_type = float(norm_type)
    mp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
    acc = torch.zeros(1, device=_dev())
    for p in parameters:
        if mp_rank == 0 or is_model_parallel_parameter(p):
            acc += p.data.float().norm(norm_type) ** norm_type
    if mpu is not None:
        dist.all_reduce(acc, group=mpu.get_model_parallel_group())
    total = acc.item() ** (1.0 / norm_type)
    if total in (float("inf"), -float("inf")) or total != total:
        total = -1
    return total


def clip_grad_norm_(parameters, max_norm, norm_type=2, mpu=None):
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = list(filter(lambda p: p.grad is not None, parameters))
    total_norm = get_grad_norm(parameters, norm_type, mpu)
    clip_coef = max_norm / (total_norm + 1e-6)
    if total_norm > 0 and clip_coef < 1:
        for p in parameters:
            p.grad.data.mul_(clip_coef)
    return total_norm


# ------------------------------------------------------------------------------ partitioning
def prefix_sum_inc(weights):
    out = []
    s = 0
    for w in weights:
        s += w
        out.append(s)
    return out


def partition_uniform(num_items, num_parts):
    """Boundaries [0, ..., num_items] of num_parts near-equal contiguous parts (the last
    part absorbs the remainder)."""
    if num_items <= num_parts:
        return [min(p, num_items) for p in range(num_parts + 1)]
    size = floor(num_items / num_parts)
    parts = [min(size * p, num_items) for p in range(num_parts)]
    parts.append(num_items)
    return parts


def _probe(prefix, num_parts, limit):
    """Greedy left-to-right cut: every part is extended while its weight stays < limit
    (prefix sums inclusive).  Returns (boundaries, fits)."""
    n = len(prefix)
    parts = [0] + [n] * num_parts
    base = 0.0
    for p in range(1, num_parts):
        cut = bisect_left(prefix, base + limit, lo=parts[p - 1])
        parts[p] = cut
        if cut == n:
            last = prefix[-1] - (prefix[parts[p - 1] - 1] if parts[p - 1] > 0 else 0)
            return parts, last < limit
        base = prefix[cut - 1] if cut > 0 else 0.0
    return parts, prefix[-1] - base <= limit


def partition_balanced(weights, num_parts, eps=1e-3):
    """Contiguous partition minimising the heaviest part (binary search on the bottleneck)."""
    if len(weights) <= num_parts:
        return partition_uniform(len(weights), num_parts)
    prefix = prefix_sum_inc(weights)
    lo, hi = prefix[-1] / num_parts, float(prefix[-1])
    while hi > lo + eps:
        mid = lo + (hi - lo) / 2
        _, ok = _probe(prefix, num_parts, mid)
        if ok:
            hi = mid
        else:
            lo = mid + eps
    parts, ok = _probe(prefix, num_parts, hi)
    assert ok
    return parts


class PartitionedTensor:
    """A tensor split evenly over a process group (tensor-parallel activation sharding for
    pipeline stage boundaries, reference runtime/utils.py:417-520)."""

    def __init__(self, tensor, group, partition_meta=None):
        self.group = group
        self.num_parts = dist.get_world_size(group=group)
        self.rank = dist.get_rank(group=group)
        self.orig_size = list(tensor.size())
        self.orig_device = tensor.device
        self.local_data, self.partition = self._partition_tensor(tensor)

    @classmethod
    def from_meta(cls, meta, local_part, group, device="cuda"):
        assert meta.dtype == torch.long
        obj = cls(tensor=torch.ones(dist.get_world_size(group=group)), group=group)
        m = meta.tolist()
        ndim = m[0]
        obj.orig_size = m[1:1 + ndim]
        m = m[1 + ndim:]
        obj.orig_device = device
        obj.local_data = local_part.detach()
        obj.group = group
        assert obj.num_parts == m[0]
        assert obj.rank == m[1]
        obj.partition = m[2:]
        return obj

    def _partition_tensor(self, tensor):
        part = partition_uniform(num_items=tensor.numel(), num_parts=self.num_parts)
        start, length = part[self.rank], part[self.rank + 1] - part[self.rank]
        local = tensor.detach().contiguous().view(-1).narrow(0, start, length).clone()
        return local, part

    def full(self, device=None):
        device = self.orig_device if device is None else device
        n = int(np.prod(self.full_size()))
        sizes = [self.partition[i + 1] - self.partition[i] for i in range(self.num_parts)]
        width = max(sizes)
        # collectives need equal-sized pieces: gather padded parts, then compact
        padded = torch.zeros(width * self.num_parts, dtype=self.local_data.dtype, device=device)
        mine = torch.zeros(width, dtype=self.local_data.dtype, device=device)
        mine[: sizes[self.rank]].copy_(self.local_data)
        dist.all_gather_into_tensor(padded, mine, group=self.group)
        if all(s == width for s in sizes):
            flat = padded[:n]
        else:
            flat = torch.cat([padded[i * width: i * width + sizes[i]] for i in range(self.num_parts)])
        return flat.view(self.full_size()).clone().detach()

    def to_meta(self):
        meta = [len(self.orig_size)] + list(self.orig_size) + [self.num_parts, self.rank] + list(self.partition)
        return torch.LongTensor(data=meta).to(self.orig_device)

    def data(self):
        return self.local_data

    def local_size(self):
        return self.local_data.size()

    def full_size(self):
        return self.orig_size


# ------------------------------------------------------------------------------ memory
mem_alloced = 0
mem_cached = 0


def memory_status(msg, print_rank=-1, reset_max=False):
    global mem_alloced, mem_cached
    rank = dist.get_rank() if dist.is_initialized() else 0
    if print_rank != -1 and rank != print_rank:
        return
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    if reset_max:
        torch.cuda.reset_peak_memory_stats()
    new_alloced = torch.cuda.memory_allocated()
    new_cached = torch.cuda.memory_reserved()
    delta_a, delta_c = new_alloced - mem_alloced, new_cached - mem_cached
    mem_alloced, mem_cached = new_alloced, new_cached
    logger.info(f"RANK={rank} MEMSTATS {msg} device={torch.cuda.current_device()} "
                f"current alloc={new_alloced / 2**30:0.4f}GB (delta={delta_a / 2**30:0.4f}GB "
                f"max={torch.cuda.max_memory_allocated() / 2**30:0.4f}GB) current cache={new_cached / 2**30:0.4f}GB "
                f"(delta={delta_c / 2**30:0.4f}GB max={torch.cuda.max_memory_reserved() / 2**30:0.4f}GB)")


def see_memory_usage(message, force=False):
    if not force:
        return
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    gc.collect()
    if torch.cuda.is_available():
        logger.info(message)
        logger.info(f"MA {round(torch.cuda.memory_allocated() / 2**30, 2)} GB "
                    f"Max_MA {round(torch.cuda.max_memory_allocated() / 2**30, 2)} GB "
                    f"CA {round(torch.cuda.memory_reserved() / 2**30, 2)} GB "
                    f"Max_CA {round(torch.cuda.max_memory_reserved() / 2**30)} GB ")
    if psutil is not None:
        vm = psutil.virtual_memory()
        logger.info(f"CPU Virtual Memory:  used = {round((vm.total - vm.available) / 2**30, 2)} GB, "
                    f"percent = {vm.percent}%")
    if torch.cuda.is_available():
        torch.cuda.reset_peak_memory_stats()


# ------------------------------------------------------------------------------ DeeperSpeed GNS
class GradientNoiseScale:
    """Gradient noise scale estimator (McCandlish et al.), DeeperSpeed runtime/utils.py:618-674.

    Every `n_batches` updates it compares |g|^2 of the current small batch with |G|^2 of the
    mean over the last n batches to estimate the true gradient norm (`scale`) and trace of
    the covariance (`noise`); both are EMA-smoothed with bias correction.
    """

    def __init__(self, model, batch_size_small, n_batches, beta):
        self.batch_size_small = batch_size_small
        self.batch_size_large = batch_size_small * n_batches
        self.n_batches = n_batches
        self.beta = beta
        self.model = model
        self.buffer = []
        self.ema_scale = None
        self.ema_noise = None
        self.scale = None
        self.noise = None
        self.noise_scale = None
        self.n_updates = 0

    def ema(self, avg, yi, i):
        avg = (0 if avg is None else avg) * self.beta + (1 - self.beta) * yi
        return avg, avg / (1 - self.beta ** (i + 1))

    def _flatten_grads(self):
        grads = [p.grad.flatten().view(-1, 1) for p in self.model.parameters() if p.grad is not None]
        return torch.cat(grads)

    def _get_scale(self, g_small, g_big):
        return (g_small - g_big) / ((1 / self.batch_size_small) - (1 / self.batch_size_large))

    def _get_noise(self, g_small, g_big):
        return (self.batch_size_large * g_big - self.batch_size_small * g_small) / (
            self.batch_size_large - self.batch_size_small)

    def update(self):
        cur = self._flatten_grads()
        self.buffer.append(cur)
        if self.n_updates % self.n_batches == self.n_batches - 1:
            past = torch.cat(self.buffer, dim=1).mean(dim=1)
            self.buffer = []
            g_big = (past ** 2).mean()
            g_small = (cur ** 2).mean()
            noise = self._get_noise(g_small, g_big)
            scale = self._get_scale(g_small, g_big)
            self.ema_scale, scale = self.ema(self.ema_scale, scale, self.n_updates)
            self.ema_noise, noise = self.ema(self.ema_noise, noise, self.n_updates)
            self.scale = scale.item()
            self.noise = noise.item()
            self.noise_scale = scale / noise
        self.n_updates += 1
