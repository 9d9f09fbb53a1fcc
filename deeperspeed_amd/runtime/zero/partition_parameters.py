"""ZeRO-3 parameter construction-time partitioning and gathering helpers.

Reference parity: deepspeed/runtime/zero/partition_parameters.py:1-1130 (`Init`,
`GatheredParameters`, `register_external_parameter`, `ZeroParamType`, `ZeroParamStatus`).

`Init` partitions every parameter as soon as the module that owns it finishes `__init__`, so a
model larger than one device never materialises: the parameter is broadcast from rank 0 (one
tensor at a time), rank r keeps elements [r*ps, (r+1)*ps) of the padded flat tensor as
`p.ds_tensor` and `p.data` becomes an empty placeholder.  The ZeRO-3 optimizer later adopts
these per-parameter partitions into its per-unit flat bucket layout
(stage3.DeepSpeedZeroOptimizer_Stage3._build_shards) one parameter at a time.

Unlike the reference, no global torch functions (`torch.empty`, `F.linear`, ...) are
monkey-patched: only `nn.Module.__init__` of module classes is wrapped while the context is
active, and everything is restored on exit.
"""

from __future__ import annotations

import functools
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ...utils.logging import logger
from .stage3 import ZeroParamStatus, ZeroParamType


def _dist_ready():
    return dist.is_available() and dist.is_initialized()


def _comm_device(t: torch.Tensor, group=None) -> torch.device:
    """Collectives on the nccl (RCCL) backend need device tensors."""
    if _dist_ready() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return t.device


def is_zero_param(p) -> bool:
    return hasattr(p, "ds_tensor") or hasattr(p, "ds_id")


def _partition_size(numel: int, world: int) -> int:
    return (numel + world - 1) // world


def _gather_full(p: torch.Tensor, group=None) -> torch.Tensor:
    """Full flat tensor of an Init-partitioned parameter (collective over `group`)."""
    world = dist.get_world_size(group) if _dist_ready() else 1
    part = p.ds_tensor
    dev = _comm_device(part, group)
    src = part.to(dev)
    if world == 1:
        return src[: p.ds_numel].clone()
    out = torch.empty(part.numel() * world, dtype=part.dtype, device=dev)
    dist.all_gather_into_tensor(out, src.contiguous(), group=group)
    return out[: p.ds_numel]


def _partition_param(p: nn.Parameter, group, remote_device, pin_memory):
    if hasattr(p, "ds_tensor"):
        return
    world = dist.get_world_size(group) if _dist_ready() else 1
    rank = dist.get_rank(group) if _dist_ready() else 0
    full = p.data
    if _dist_ready() and world > 1:
        dev = _comm_device(full, group)
        t = full.to(dev).contiguous()
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        full = t
    flat = full.reshape(-1)
    ps = _partition_size(flat.numel(), world)
    part = torch.zeros(ps, dtype=flat.dtype, device=flat.device)
    lo, hi = rank * ps, min(flat.numel(), (rank + 1) * ps)
    if hi > lo:
        part[: hi - lo].copy_(flat[lo:hi])
    target = torch.device(remote_device) if remote_device not in (None, "none") else p.device
    if target.type == "cpu":
        part = part.cpu()
        if pin_memory and torch.cuda.is_available():
            part = part.pin_memory()
    else:
        part = part.to(target)
    p.ds_tensor = part
    p.ds_numel = flat.numel()
    p.ds_shape = p.shape
    p.ds_status = ZeroParamStatus.NOT_AVAILABLE
    p.ds_persist = False
    p.ds_process_group = group
    p.data = torch.empty(0, dtype=p.dtype, device=p.device)
    _attach_methods(p)


def _attach_methods(p):
    """Per-parameter helpers mirroring the reference's `param.all_gather()` / `partition()`."""

    def all_gather(param_list=None, async_op=False):
        for q in (param_list or [p]):
            if q.ds_status == ZeroParamStatus.NOT_AVAILABLE:
                full = _gather_full(q, q.ds_process_group)
                q.data = full.view(q.ds_shape).to(q.ds_tensor.device if q.ds_tensor.is_cuda else full.device)
                q.ds_status = ZeroParamStatus.AVAILABLE
        return None

    def partition(param_list=None, has_been_updated=False):
        for q in (param_list or [p]):
            if q.ds_status != ZeroParamStatus.AVAILABLE:
                continue
            if has_been_updated:
                world = dist.get_world_size(q.ds_process_group) if _dist_ready() else 1
                rank = dist.get_rank(q.ds_process_group) if _dist_ready() else 0
                flat = q.data.reshape(-1)
                ps = q.ds_tensor.numel()
                lo, hi = rank * ps, min(flat.numel(), (rank + 1) * ps)
                q.ds_tensor.zero_()
                if hi > lo:
                    q.ds_tensor[: hi - lo].copy_(flat[lo:hi].to(q.ds_tensor.device))
            q.data = torch.empty(0, dtype=q.dtype, device=q.device)
            q.ds_status = ZeroParamStatus.NOT_AVAILABLE

    def padding_size():
        world = dist.get_world_size(p.ds_process_group) if _dist_ready() else 1
        return p.ds_tensor.numel() * world - p.ds_numel

    p.all_gather = all_gather
    p.partition = partition
    p.padding_size = padding_size
    p.ds_summary = lambda: dict(id=id(p), status=p.ds_status, numel=p.ds_numel, shape=tuple(p.ds_shape),
                                partition=p.ds_tensor.numel())


class Init:
    """Context manager / decorator partitioning parameters at module construction.

        with deeperspeed_amd.zero.Init(data_parallel_group=group, remote_device="cpu"):
            model = BigModel()
    """

    def __init__(self, module=None, data_parallel_group=None, mem_efficient_linear=True, remote_device=None,
                 pin_memory=False, config=None, enabled=True, dtype=None):
        self.group = data_parallel_group
        self.remote_device = remote_device
        self.pin_memory = pin_memory
        self.enabled = enabled
        self.mem_efficient_linear = mem_efficient_linear
        self.dtype = dtype
        self._patched = []
        if module is not None and enabled:
            # convert an existing module in place
            for m in module.modules():
                for p in m.parameters(recurse=False):
                    _partition_param(p, self.group, self.remote_device, self.pin_memory)

    def _wrap(self, cls):
        orig = cls.__dict__.get("__init__")
        if orig is None or getattr(orig, "_dsa_zero_init", False):
            return
        ctx = self

        @functools.wraps(orig)
        def wrapped(module, *args, **kwargs):
            orig(module, *args, **kwargs)
            # only the most-derived __init__ partitions (base-class __init__s run first)
            if type(module).__init__ is wrapped or type(module).__dict__.get("__init__") is wrapped:
                for p in module.parameters(recurse=False):
                    if ctx.dtype is not None and p.dtype.is_floating_point:
                        p.data = p.data.to(ctx.dtype)
                    _partition_param(p, ctx.group, ctx.remote_device, ctx.pin_memory)

        wrapped._dsa_zero_init = True
        cls.__init__ = wrapped
        self._patched.append((cls, orig))

    def _all_module_classes(self):
        seen, stack = set(), [nn.Module]
        while stack:
            c = stack.pop()
            for s in c.__subclasses__():
                if s not in seen:
                    seen.add(s)
                    stack.append(s)
        return seen

    def __enter__(self):
        if not self.enabled:
            return self
        for cls in self._all_module_classes():
            self._wrap(cls)
        self._orig_init_subclass = nn.Module.__dict__.get("__init_subclass__")
        ctx = self

        def init_subclass(cls, **kw):
            super(nn.Module, cls).__init_subclass__(**kw)
            ctx._wrap(cls)

        nn.Module.__init_subclass__ = classmethod(init_subclass)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        for cls, orig in reversed(self._patched):
            cls.__init__ = orig
        self._patched = []
        if self._orig_init_subclass is None:
            del nn.Module.__init_subclass__
        else:
            nn.Module.__init_subclass__ = self._orig_init_subclass
        return False

    def __call__(self, fn):
        @functools.wraps(fn)
        def inner(*a, **kw):
            with self:
                return fn(*a, **kw)

        return inner


class GatheredParameters:
    """Temporarily materialise ZeRO-3 parameters (Init-partitioned or engine-owned).

    With `modifier_rank=r`, rank r's edits are broadcast and written back into every rank's
    partition (and the fp32 master) on exit."""

    def __init__(self, params, modifier_rank: Optional[int] = None, fwd_module=None, enabled: bool = True):
        if isinstance(params, nn.Parameter) or torch.is_tensor(params):
            params = [params]
        self.params: List[nn.Parameter] = [p for p in params if is_zero_param(p)]
        self.modifier_rank = modifier_rank
        self.enabled = enabled and bool(self.params)
        self._units = []
        self._was_single = False

    def __enter__(self):
        if not self.enabled:
            return self
        owner = getattr(self.params[0], "_ds_owner", None)
        if owner is not None:  # engine-owned: fetch the units
            self._owner = owner
            seen = []
            for p in self.params:
                u = owner.unit_of(p)
                if u is not None and u not in seen:
                    seen.append(u)
            self._was = [u.status for u in seen]
            self._units = seen
            owner.gather_units(seen)
        else:
            self._owner = None
            for p in self.params:
                p.all_gather()
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        if self.modifier_rank is not None and _dist_ready():
            for p in self.params:
                t = p.data.to(_comm_device(p.data)).contiguous()
                dist.broadcast(t, src=self.modifier_rank)
                p.data.copy_(t.to(p.data.device))
        if self._owner is not None:
            if self.modifier_rank is not None:
                self._owner.write_back_params(self.params)
            for u, was in zip(self._units, self._was):
                if was == ZeroParamStatus.NOT_AVAILABLE:
                    self._owner.release_units([u], force=True)
        else:
            for p in self.params:
                p.partition(has_been_updated=self.modifier_rank is not None)
        return False


def register_external_parameter(module: nn.Module, parameter: nn.Parameter):
    """Declare that `module.forward` uses `parameter` although it belongs to another module,
    so ZeRO-3 gathers it whenever `module` runs (reference partition_parameters.py:46-96)."""
    if not isinstance(parameter, nn.Parameter):
        raise RuntimeError("Parameter is not a torch.nn.Parameter")
    lst = module.__dict__.setdefault("_external_params", [])
    if all(q is not parameter for q in lst):
        lst.append(parameter)
    owner = getattr(parameter, "_ds_owner", None)
    if owner is not None:
        owner.register_external_parameter(module, parameter)
