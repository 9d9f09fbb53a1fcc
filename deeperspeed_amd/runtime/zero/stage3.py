"""ZeRO stage 3: parameter + gradient + optimizer-state partitioning.

Reference parity (behaviour): deepspeed/runtime/zero/stage3.py (module pre/post forward and
backward hooks, trace-driven prefetch bounded by `stage3_prefetch_bucket_size`, persistent
small parameters below `stage3_param_persistence_threshold`, per-bucket gradient
reduce-scatter during backward, sub-group steps, ZeRO-Offload / Infinity of optimizer
state) and partition_parameters.py (`ds_shape`, `ds_numel`, status, external params).

MI355X design:
* Parameters are grouped into *units* (a module subtree of at most
  `stage3_unit_max_numel` elements, else its direct params); each (unit, param group) is
  ONE flat bucket.  Gathering a unit = one `all_gather_into_tensor` per bucket straight
  into a fresh flat buffer whose slices become the parameters' storage; releasing drops
  the buffer back to the caching allocator.  Gradient reduction = one
  `reduce_scatter_tensor` per bucket as soon as the unit's backward completes.
* Collectives are asynchronous on RCCL's stream; compute waits with stream-level
  `work.wait()` only right before the unit is used (no device-wide synchronize).
* Prefetch follows the forward/backward unit order recorded on the first step.
* With a data-parallel world of 1 the shard IS the full parameter: parameters are bound
  to views of the shard permanently and gradients accumulate in place into the shard
  gradient (no gather, no copy) -- this is what makes the single-GPU 20B path fit in HBM.
"""

from __future__ import annotations

import functools
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ...utils.logging import logger
from ...utils import comm
from .layout import ALIGN, FlatGroup, build_unit_buckets
from .sharded_base import ShardedOptimizerBase, _dist_ready

OVERLAP_TRACE = False  # log each overlapped-step bucket wait (diagnostics)


class ZeroParamStatus:
    AVAILABLE = 1
    NOT_AVAILABLE = 2
    INFLIGHT = 3


class ZeroParamType:
    NORMAL = 1
    PARTITIONED = 2
    REMOTE = 3


_EMPTY: Dict = {}


def _empty_like(dtype, device):
    key = (dtype, device)
    t = _EMPTY.get(key)
    if t is None:
        t = torch.empty(0, dtype=dtype, device=device)
        _EMPTY[key] = t
    return t


def _numel(p):
    return p.ds_numel if hasattr(p, "ds_tensor") else p.numel()


def _in_backward():
    return torch._C._current_graph_task_id() != -1


class _BufferPool:
    """Persistent device buffers for gathered units and unit gradients.

    RCCL collectives record their tensors on the communicator's stream, so a buffer freed
    back to the caching allocator only becomes reusable once that stream's event has
    completed; with the host running ahead of the GPU the allocator keeps growing.  Buffers
    returned here are reused immediately: later work on the compute stream is
    stream-ordered after their last use, and ProcessGroupNCCL makes its stream wait for the
    compute stream before each collective, so a reused buffer never races an earlier
    reader.  Sizes are rounded up to `SIZE_CLASS` elements so units of nearly equal size
    (GPT-NeoX attention / MLP-in / MLP-out are all ~151M elements at 20B) share buffers."""

    SIZE_CLASS = 1 << 22

    def __init__(self):
        self.free: Dict[tuple, List[torch.Tensor]] = {}
        self.held = 0  # elements owned by the pool (free + handed out)

    def _cls(self, numel):
        return -(-int(numel) // self.SIZE_CLASS) * self.SIZE_CLASS if numel > self.SIZE_CLASS else int(numel)

    def get(self, numel, dtype, device, zero=False):
        c = self._cls(numel)
        lst = self.free.get((dtype, c, str(device)))
        if lst:
            base = lst.pop()
        else:
            self.held += c
            base = torch.empty(c, dtype=dtype, device=device)
        t = base[:numel] if c != numel else base
        if zero:
            t.zero_()
        return t

    def put(self, t):
        base = t if t._base is None else t._base
        self.free.setdefault((base.dtype, base.numel(), str(base.device)), []).append(base)

    def clear(self):
        for lst in self.free.values():
            self.held -= sum(t.numel() for t in lst)
        self.free = {}


class ZeroUnit:
    def __init__(self, uid, module, params):
        self.uid = uid
        self.module = module
        self.params = list(params)
        self.buckets = []  # (FlatGroup, Bucket)
        self.status = ZeroParamStatus.NOT_AVAILABLE
        self.works = []
        self.fulls = []
        self.numel = sum(_numel(p) for p in self.params)
        self.persistent = False
        self.active = 0
        self.in_backward = False
        self.grad_fulls = []
        self.bw_expected = 0
        self.bw_ready = 0
        self.reduced = False
        self.external = []  # units whose params this module also uses (register_external_parameter)

    def __repr__(self):
        return f"ZeroUnit({self.uid}, {type(self.module).__name__}, numel={self.numel})"


class DeepSpeedZeroOptimizer_Stage3(ShardedOptimizerBase):
    def __init__(self, module, init_optimizer, dp_process_group=None, mpu=None, clip_grad=0.0,
                 static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None,
                 prefetch_bucket_size=int(5e7), max_live_parameters=int(1e9), max_reuse_distance=int(1e9),
                 param_persistence_threshold=int(1e5), unit_max_numel=int(2e8), fp32_reduce=False,
                 gradient_predivide_factor=1.0, gradient_accumulation_steps=1, offload_optimizer=None,
                 offload_param=None, timers=None, overlap_comm=True, sub_group_size=int(1e12), verbose=False,
                 compact_master=False, force_sharded=False, resident_grads=False, grad_accum_dtype="auto",
                 reduce_scatter=True, reduce_bucket_size=0, overlap_step=False):
        super().__init__(init_optimizer, dp_process_group=dp_process_group, mpu=mpu, clip_grad=clip_grad,
                         static_loss_scale=static_loss_scale, dynamic_loss_scale=dynamic_loss_scale,
                         dynamic_loss_args=dynamic_loss_args, fp32_reduce=fp32_reduce,
                         gradient_predivide_factor=gradient_predivide_factor,
                         gradient_accumulation_steps=gradient_accumulation_steps,
                         offload_optimizer=offload_optimizer, timers=timers, verbose=verbose,
                         compact_master=compact_master, sub_group_size=sub_group_size)
        self.module = module
        self.stage = 3
        # overlap_comm=False (reference stage3.py:706,826): collectives are waited for right
        # where they are issued and nothing is prefetched
        self.overlap_comm = True if overlap_comm is None else bool(overlap_comm)
        # reduce_scatter=False (reference stage3.py:1948): gradients are all-reduced per bucket
        # and each rank keeps its chunk -- twice the traffic, kept for parity only
        self.use_reduce_scatter = bool(reduce_scatter)
        # in-flight gradient reductions are bounded (sharded_base._queue_reduction): at most
        # two reduce buckets' worth, or two units when units are larger
        self.max_inflight_numel = 2 * int(reduce_bucket_size or 0)
        # MI355X extension: run the sharded gather / reduce-scatter machinery even on a world of
        # one (the real RCCL code path of N>1, on one GPU) instead of binding params to shards
        self.force_sharded = bool(force_sharded)
        # MI355X extension: keep each unit's full gradient buffer resident across the
        # micro-batches of one optimizer step and reduce-scatter once, at the accumulation
        # boundary (GA x fewer reduce-scatters; costs one bf16 copy of the model's gradients)
        self.resident_grads = bool(resident_grads)
        self.grad_accum_dtype = str(grad_accum_dtype or "auto")
        self.prefetch_bucket_size = int(prefetch_bucket_size)
        self.max_live_parameters = int(max_live_parameters)
        self.max_reuse_distance = int(max_reuse_distance)
        self.persistence_threshold = int(param_persistence_threshold)
        self.unit_max_numel = int(unit_max_numel)
        self.offload_param = offload_param
        # ZeRO-Infinity parameter offload: bf16 shards in pinned host memory ("cpu") or in a
        # file-backed mapping on the NVMe path ("nvme"); every fetch stages the unit's chunk to
        # HBM before the all-gather, the (offloaded) optimizer writes updated shards back.
        self.param_offload = bool(offload_param) and offload_param.get("device") in ("cpu", "nvme")
        if self.param_offload and self.offload is None:
            raise ValueError("offload_param requires offload_optimizer (cpu or nvme) in ZeRO stage 3")
        # "nvme": the shard lives only in per-(group, bucket) files behind the aio engine
        # (runtime/swap_tensor/partitioned_param_swapper.py); "mmap" keeps the older file-backed
        # mapping through the page cache
        self.param_nvme = self.param_offload and offload_param.get("device") == "nvme" and \
            offload_param.get("mode", "aio") == "aio"
        if self.param_nvme and self.offload_states == "master" and not self.nvme:
            raise ValueError("offload_param nvme needs the optimizer step on the host (offload_optimizer states 'all' or nvme)")
        self._pswap = None
        self._pkey: Dict[int, tuple] = {}
        self.compute_device = self.device
        self.single = self.dp_world == 1 and not self.param_offload and not self.force_sharded
        if self.single:
            self.resident_grads = False  # gradients accumulate in the bound shard already
        self._pending = []
        self._fwd_trace: List[int] = []
        self._bwd_trace: List[int] = []
        self._trace_frozen = False
        self._fwd_pos = 0
        self._bwd_pos = 0
        self._units: List[ZeroUnit] = []
        self._unit_of_param: Dict[int, ZeroUnit] = {}
        # gathered-parameter retention (reference stage3_max_live_parameters /
        # stage3_max_reuse_distance): live numel of non-persistent gathered units and the
        # per-trace-position distance (in elements) to each unit's next use
        self._live_numel = 0
        self._pool = _BufferPool()
        self.pool_skipped = 0  # released buffers still referenced elsewhere (left to the allocator)
        self.gathered_numel = 0  # elements all-gathered so far (stats / tests)
        self._reuse_f: Dict[int, int] = {}
        self._reuse_b: Dict[int, int] = {}
        self._assign_units(module)
        self.groups = self._split_groups()
        for g in self.groups:
            build_unit_buckets(g, self.dp_world, lambda p: self._unit_of_param[id(p)])
            for b in g.buckets:
                b.unit.buckets.append((g, b))
        self._build_shards()
        self._alloc_master_and_state(lambda g: g.shard_param.float())
        if self.param_nvme:
            for g in self.groups:
                g.shard_param = None  # the NVMe files are the only copy from here on
        self._register_hooks()
        self._setup_overlap_step(bool(overlap_step))
        for m in module.modules():
            for p in m.__dict__.get("_external_params", []):
                self.register_external_parameter(m, p)
        if verbose:
            n = sum(u.numel for u in self._units)
            logger.info(f"ZeRO-3: {len(self._units)} units, {n / 1e9:.3f}B params, dp_world={self.dp_world}, "
                        f"persistent units={sum(u.persistent for u in self._units)}")

    # ------------------------------------------------------------------ units
    def _assign_units(self, root):
        seen = set()

        def subtree_params(m):
            return [p for p in m.parameters() if id(p) not in seen]

        def make(m, params):
            params = [p for p in params if id(p) not in seen]
            if not params:
                return
            u = ZeroUnit(len(self._units), m, params)
            for p in params:
                seen.add(id(p))
                self._unit_of_param[id(p)] = u
            self._units.append(u)
            m._zero_unit = u

        def visit(m):
            sub = subtree_params(m)
            if not sub:
                return
            n = sum(_numel(p) for p in sub)
            kids = [c for c in m.children() if any(True for _ in c.parameters())]
            if n <= self.unit_max_numel or not kids:
                make(m, sub)
                return
            for c in m.children():
                visit(c)
            make(m, list(m.parameters(recurse=False)))

        visit(root)
        # module -> unit whose hooks run around it (nearest ancestor unit root)
        self._unit_of_module = {}

        def label(m, cur):
            cur = getattr(m, "_zero_unit", None) or cur
            self._unit_of_module[id(m)] = cur
            for c in m.children():
                label(c, cur)

        label(root, None)
        for u in self._units:
            u.persistent = u.numel <= self.persistence_threshold and not self.single
            for p in u.params:
                if not hasattr(p, "ds_tensor"):  # zero.Init params carry their full shape
                    p.ds_numel = p.numel()
                    p.ds_shape = p.shape
                p.ds_id = id(p)
                p.ds_unit = u
                p.ds_status = ZeroParamStatus.AVAILABLE

    def _build_shards(self):
        """Create per-group bf16 shards from the (currently full) parameters, then free them."""
        r = self.dp_rank
        for gi, g in enumerate(self.groups):
            dev = g.params[0].device if g.params[0].is_cuda else self.device
            self.compute_device = dev
            g.shard_param = self._alloc_param_shard(gi, g, dev)
            for b in g.buckets:
                for i, p in enumerate(b.params):
                    ov = b.chunk_overlap(r, i)
                    src = p.data.reshape(-1)
                    if src.numel() == 0 and hasattr(p, "ds_tensor"):
                        # zero.Init partition: re-layout one parameter at a time (collective,
                        # every rank walks the same bucket order)
                        from .partition_parameters import _gather_full
                        src = _gather_full(p, self.dp_group)
                    if ov is None:
                        continue
                    p0, c0, ln = ov
                    g.shard_param[b.shard_offset + c0: b.shard_offset + c0 + ln].copy_(src[p0: p0 + ln])
            gdt = self._grad_dtype(g)
            g.shard_grad = torch.zeros(g.shard_numel, dtype=gdt, device=dev)
        if self.param_nvme:
            import os
            from ..swap_tensor.partitioned_param_swapper import AsyncPartitionedParameterSwapper
            folder = os.path.join(self.offload_param.get("nvme_path") or "/tmp/deeperspeed_amd_nvme", "zero_stage_3",
                                  f"params_rank{self.dp_rank}_mp{self.mp_rank}")
            self._pswap = AsyncPartitionedParameterSwapper(folder, self.groups[0].dtype if self.groups else torch.bfloat16,
                                                           buffer_count=self.offload_param.get("buffer_count", 5),
                                                           aio_config=self.offload_param.get("aio"))
            for gi, g in enumerate(self.groups):
                for bi, b in enumerate(g.buckets):
                    self._pkey[id(b)] = (gi, bi)
                    self._pswap.register((gi, bi), g.shard_param[b.shard_offset: b.shard_offset + b.chunk])
        for u in self._units:
            for p in u.params:
                p._ds_owner = self
                if hasattr(p, "ds_tensor"):
                    del p.ds_tensor  # adopted into the flat shard layout
        # release full parameters / bind permanently (single rank)
        for u in self._units:
            for g, b in u.buckets:
                for i, p in enumerate(b.params):
                    if self.single:
                        off = b.shard_offset + b.offsets[i]
                        p.data = g.shard_param[off: off + b.numels[i]].view(p.ds_shape)
                        p.grad = g.shard_grad[off: off + b.numels[i]].view(p.ds_shape)
                    else:
                        p.data = _empty_like(g.dtype, self.compute_device)
            u.status = ZeroParamStatus.AVAILABLE if self.single else ZeroParamStatus.NOT_AVAILABLE
        if not self.single:
            for u in self._units:
                if u.persistent:
                    self._fetch(u)
                    self._wait(u)
        if torch.cuda.is_available():
            torch.cuda.empty_cache()

    def _alloc_param_shard(self, gi, g, dev):
        if not self.param_offload:
            return torch.zeros(g.shard_numel, dtype=g.dtype, device=dev)
        if self.param_nvme:
            return torch.zeros(g.shard_numel, dtype=g.dtype)  # staging for init, dropped after
        if self.offload_param.get("device") == "nvme":
            import os
            folder = os.path.join(self.offload_param.get("nvme_path") or "/tmp/deeperspeed_amd_nvme", "zero_stage_3",
                                  f"params_rank{self.dp_rank}_mp{self.mp_rank}")
            os.makedirs(folder, exist_ok=True)
            path = os.path.join(folder, f"group{gi}.swp")
            if os.path.exists(path):
                os.remove(path)
            t = torch.from_file(path, shared=True, size=max(1, g.shard_numel), dtype=g.dtype)[:g.shard_numel]
            t.zero_()
            return t
        pin = bool(self.offload_param.get("pin_memory", True)) and torch.cuda.is_available()
        if pin:
            from ...ops import native
            return native.pinned_zeros(g.shard_numel, g.dtype)  # exact size, not a power of two
        return torch.zeros(g.shard_numel, dtype=g.dtype)

    def _grad_dtype(self, g):
        """dtype of the reduced gradient shard (where micro-batch reductions accumulate)."""
        if self.single:
            return g.dtype  # accumulate in place (p.grad views need the param dtype)
        if self.fp32_reduce or g.dtype == torch.float32 or self.grad_accum_dtype in ("fp32", "float32"):
            return torch.float32
        if self.grad_accum_dtype != "auto":
            return g.dtype
        # auto: with resident unit grads the shard receives one reduction per step
        if self.gradient_accumulation_steps > 1 and not self.resident_grads:
            return torch.float32
        return g.dtype

    def _unit_grad_dtype(self, g):
        """dtype of a unit's full (pre-reduction) gradient buffer: autograd accumulates into it
        through the p.grad views, so it is the parameter dtype (resident micro-batch sums too)."""
        return g.dtype

    def _collective(self):
        return _dist_ready() and (self.dp_world > 1 or self.force_sharded)

    # ------------------------------------------------------------------ gather / release
    def _fetch(self, u: ZeroUnit):
        if u.status != ZeroParamStatus.NOT_AVAILABLE:
            return
        u.works, u.fulls = [], []
        if not u.persistent:
            self._live_numel += u.numel
        self.gathered_numel += u.numel
        for g, b in u.buckets:
            full = self._pool.get(b.numel, g.dtype, self.compute_device)
            if self.param_nvme and g.shard_param is None:
                chunk = self._pswap.read_to_device(self._pkey[id(b)], self.compute_device)
            else:
                chunk = g.shard_param[b.shard_offset: b.shard_offset + b.chunk]
                if self.param_offload:
                    chunk = chunk.to(self.compute_device, non_blocking=chunk.is_pinned())
            if self._collective():
                w = comm.all_gather_into_tensor(full, chunk, group=self.dp_group, async_op=True,
                                                tag=f"zero3.gather.u{u.uid}")
                if self.overlap_comm:
                    u.works.append(w)
                else:
                    w.wait()
            else:
                full.copy_(chunk)
            u.fulls.append(full)
            for i, p in enumerate(b.params):
                p.data = full[b.offsets[i]: b.offsets[i] + b.numels[i]].view(p.ds_shape)
                p.ds_status = ZeroParamStatus.INFLIGHT
        u.status = ZeroParamStatus.INFLIGHT

    def _wait(self, u: ZeroUnit):
        if u.status == ZeroParamStatus.INFLIGHT:
            for w in u.works:
                w.wait()
            u.works = []
            if comm.DEBUG:
                for full in u.fulls:
                    comm.check_replicated(full, self.dp_group, f"zero3 unit {u.uid} gathered bucket")
            u.status = ZeroParamStatus.AVAILABLE
            for p in u.params:
                p.ds_status = ZeroParamStatus.AVAILABLE

    def _release(self, u: ZeroUnit, force=False):
        if self.single or u.status == ZeroParamStatus.NOT_AVAILABLE:
            return
        if u.persistent and not force:
            return
        if u.status == ZeroParamStatus.INFLIGHT:
            self._wait(u)
        for g, b in u.buckets:
            e = _empty_like(g.dtype, self.compute_device)
            for p in b.params:
                p.data = e
                p.ds_status = ZeroParamStatus.NOT_AVAILABLE
        for full in u.fulls:
            # a gathered buffer still referenced elsewhere (e.g. a view autograd saved for
            # backward) goes back to the allocator instead; it must not be overwritten
            if _sole_owner(full):
                self._pool.put(full)
            else:
                self.pool_skipped += 1
        u.fulls = []
        u.status = ZeroParamStatus.NOT_AVAILABLE
        if not u.persistent:
            self._live_numel -= u.numel

    def _compute_reuse(self):
        """Distance (in parameter elements) from each trace position to the unit's next use,
        cyclic over one micro-batch (forward trace then backward trace)."""
        order = [u for u in self._fwd_trace] + [u for u in self._bwd_trace]
        n, nf = len(order), len(self._fwd_trace)
        numel = [self._units[uid].numel for uid in order]
        self._reuse_f, self._reuse_b = {}, {}
        for i, uid in enumerate(order):
            d = 0
            for k in range(1, n + 1):
                j = (i + k) % n
                if order[j] == uid:
                    break
                d += numel[j]
            if i < nf:
                self._reuse_f[i] = d
            else:
                self._reuse_b[i - nf] = d

    def _maybe_release(self, u: ZeroUnit, phase: str):
        """Release after use unless the unit is reused within stage3_max_reuse_distance and the
        live-parameter budget (stage3_max_live_parameters) still has room."""
        if self.single or u.persistent or not self._trace_frozen:
            self._release(u)
            return
        pos = getattr(u, "last_fpos" if phase == "f" else "last_bpos", None)
        d = (self._reuse_f if phase == "f" else self._reuse_b).get(pos)
        if d is not None and d <= self.max_reuse_distance and self._live_numel <= self.max_live_parameters:
            return
        self._release(u)

    def gather_units(self, units):
        for u in units:
            self._fetch(u)
        for u in units:
            self._wait(u)

    def release_units(self, units, force=False):
        for u in units:
            self._release(u, force=force)

    def unit_of(self, p) -> Optional[ZeroUnit]:
        return self._unit_of_param.get(id(p))

    # ------------------------------------------------------------------ overlapped step
    # MI355X extension (`zero_optimization.overlap_step`, bound single-rank path): the fused
    # Adam of one optimizer step runs on a side stream, bucket by bucket, while the next
    # forward starts on the compute stream; each module's forward pre-hook waits only for the
    # event of the bucket(s) holding its own parameters, so layer 0 resumes after the first
    # bucket's update instead of after the whole step (HBM-bound Adam next to compute-bound
    # GEMMs).  Gradients are zeroed on the side stream after their update, and the next
    # backward (and every state access: checkpoints, zero_grad, ...) first waits for the whole
    # step.  Parameters read outside a module forward right after step() need
    # `synchronize_step()` (the engine calls it before checkpointing).
    def _setup_overlap_step(self, enabled: bool):
        self._overlap_step = (enabled and self.single and self.offload is None and self.fused
                              and torch.cuda.is_available() and str(self.device).startswith("cuda"))
        self._step_stream = None
        self._step_done = None
        self._bucket_events: Dict[tuple, torch.cuda.Event] = {}
        if not self._overlap_step:
            return
        from ..overlap_step import new_stream
        self._step_stream = new_stream(self.device)
        self._bucket_key = {}
        owner = {}
        for gi, g in enumerate(self.groups):
            for bi, b in enumerate(g.buckets):
                self._bucket_key[id(b)] = (gi, bi)
                for p in b.params:
                    owner[id(p)] = (gi, bi)
        self._module_buckets = {}
        for m in self.module.modules():
            # a parameter registered in several modules (tied weights) is waited for by each
            keys = sorted({owner[id(p)] for p in m.parameters(recurse=False) if id(p) in owner})
            if keys:
                self._module_buckets[m] = keys
                self._handles.append(m.register_forward_pre_hook(self._wait_bucket_updates))
        # Parameters whose owning module's forward never runs (read by a parent or a sibling:
        # F.linear(x, self.embed.weight), parameter containers) have no hook of their own.  The
        # first overlapped forward waits for the WHOLE step at the root and records which
        # modules' pre-hooks fire; from then on the root waits for the buckets of every module
        # that did not fire.  (A parameter read before its own module's forward in the same
        # pass still needs synchronize_step(): waits are stream-ordered, so any read after the
        # owner's forward is safe.)
        self._fired = set()
        self._uncovered = None  # bucket keys the root waits for; None = not calibrated yet
        self._handles.append(self.module.register_forward_pre_hook(self._root_wait_uncovered))

    def _trace_wait(self, what, key):
        """OVERLAP_TRACE = True: log each bucket wait of the first forward after a step, with the
        position of that bucket's update in the step (how much of the step the forward waits for)."""
        if not OVERLAP_TRACE:
            return
        order = list(self._bucket_events)
        pos = order.index(key) if key in order else -1
        logger.info(f"overlap_step wait: {what} bucket {key} = update {pos + 1} of {len(order)}")

    def _root_wait_uncovered(self, module, inputs):
        if not self._bucket_events or _in_backward():
            return
        cur = torch.cuda.current_stream()
        if self._uncovered is None:
            cur.wait_event(self._step_done_event)  # calibration pass: the whole step
            if OVERLAP_TRACE:
                logger.info("overlap_step wait: calibration pass waits for the whole step")
            self._calibrating = True
            self._fired = set()
            return
        for key in self._uncovered:
            ev = self._bucket_events.get(key)
            if ev is not None:
                self._trace_wait("root (uncovered)", key)
                cur.wait_event(ev)

    def _wait_bucket_updates(self, module, inputs):
        if getattr(self, "_calibrating", False):
            self._fired.add(module)
        if not self._bucket_events:
            return
        cur = torch.cuda.current_stream()
        for key in self._module_buckets.get(module, ()):
            ev = self._bucket_events.get(key)
            if ev is not None:
                self._trace_wait(type(module).__name__, key)
                cur.wait_event(ev)

    def _finish_calibration(self):
        if getattr(self, "_calibrating", False):
            self._calibrating = False
            self._uncovered = sorted({k for m, keys in self._module_buckets.items() if m not in self._fired
                                      for k in keys})
            if OVERLAP_TRACE:
                logger.info(f"overlap_step calibrated: {len(self._fired)} modules fired, root waits for "
                            f"{len(self._uncovered)} uncovered bucket(s) {self._uncovered[:8]}")

    def synchronize_step(self):
        """Order the compute stream after an overlapped optimizer step (no host wait)."""
        if self._overlap_step:
            self._finish_calibration()
        if self._step_done is not None:
            torch.cuda.current_stream().wait_event(self._step_done)
            self._step_done = None
            self._bucket_events = {}

    def step(self, closure=None):
        if not self._overlap_step:
            return super().step(closure)
        self.synchronize_step()
        overflow, total = self._check_overflow_and_scale()  # host sync: the gradients are final
        if overflow:
            self.zero_grad()
            return
        grad_scale, _ = self._unscale_and_clip_coef(total)
        side, cur = self._step_stream, torch.cuda.current_stream()
        side.wait_stream(cur)
        self._bucket_events = {}
        with torch.cuda.stream(side):
            self._inner_step(grad_scale)
            self._post_step()
            for g in self.groups:  # each bucket's gradients after its update, on the same stream
                g.shard_grad.zero_()
            self._grads_nonzero = False
        self._step_done = torch.cuda.Event()
        self._step_done.record(side)
        self._step_done_event = self._step_done

    # ------------------------------------------------------------------ hooks
    def _register_hooks(self):
        self._handles = []
        if self.single:
            return  # parameters are permanently materialised; grads land in place
        root = self.module
        self._handles.append(root.register_forward_pre_hook(self._root_pre_forward))
        for u in self._units:
            m = u.module
            self._handles.append(m.register_forward_pre_hook(functools.partial(self._pre_forward, u)))
            self._handles.append(m.register_forward_hook(functools.partial(self._post_forward, u)))
            for p in u.params:
                if p.requires_grad:
                    self._handles.append(p.register_post_accumulate_grad_hook(self._grad_ready))

    def _root_pre_forward(self, module, inputs):
        if not _in_backward():
            self._fwd_pos = 0

    def _prefetch(self, trace, pos):
        if not self._trace_frozen or pos < 0 or not self.overlap_comm:
            return
        # the window is the next `prefetch_bucket_size` elements of the trace, counting units
        # already gathered or in flight: a budget charged only for new fetches would let every
        # pre-forward hook push the frontier one unit further until the whole model is gathered
        budget = self.prefetch_bucket_size
        k = pos + 1
        seen = set()
        while k < len(trace) and budget > 0:
            u = self._units[trace[k]]
            k += 1
            if u.persistent or u.uid in seen:
                continue
            seen.add(u.uid)
            budget -= u.numel
            if u.status == ZeroParamStatus.NOT_AVAILABLE:
                self._fetch(u)

    def _pre_forward(self, u: ZeroUnit, module, inputs):
        u.active += 1
        if not _in_backward():
            if not self._trace_frozen:
                self._fwd_trace.append(u.uid)
            elif self._fwd_pos < len(self._fwd_trace) and self._fwd_trace[self._fwd_pos] == u.uid:
                self._prefetch(self._fwd_trace, self._fwd_pos)
            u.last_fpos = self._fwd_pos
            self._fwd_pos += 1
        self._fetch(u)
        for x in u.external:
            self._fetch(x)
        self._wait(u)
        for x in u.external:
            self._wait(x)

    def _post_forward(self, u: ZeroUnit, module, inputs, output):
        u.active -= 1
        if torch.is_grad_enabled():
            self._register_bw_hooks(u, output)
        if u.active == 0 and not _in_backward():
            self._maybe_release(u, "f")
            for x in u.external:
                if x.active == 0:
                    self._release(x)
        return None

    def _register_bw_hooks(self, u, output):
        def visit(o):
            if torch.is_tensor(o):
                if o.requires_grad and o.grad_fn is not None:
                    o.register_hook(functools.partial(self._pre_backward_hook, u))
            elif isinstance(o, (list, tuple)):
                for x in o:
                    visit(x)
            elif isinstance(o, dict):
                for x in o.values():
                    visit(x)
        visit(output)

    def _pre_backward_hook(self, u, grad):
        self._pre_backward(u)
        return None

    def _pre_backward(self, u: ZeroUnit):
        if u.in_backward or u.reduced:
            return
        if not self._trace_frozen:
            self._bwd_trace.append(u.uid)
        elif self._bwd_pos < len(self._bwd_trace) and self._bwd_trace[self._bwd_pos] == u.uid:
            self._prefetch(self._bwd_trace, self._bwd_pos)
        u.last_bpos = self._bwd_pos
        self._bwd_pos += 1
        self._fetch(u)
        self._wait(u)
        u.in_backward = True
        u.bw_expected = sum(1 for p in u.params if p.requires_grad)
        u.bw_ready = 0
        if not u.grad_fulls:  # resident buffers of earlier micro-batches accumulate on
            u.grad_fulls = [self._pool.get(b.numel, self._unit_grad_dtype(g), self.compute_device, zero=True)
                            for g, b in u.buckets]
        for (g, b), gf in zip(u.buckets, u.grad_fulls):
            for i, p in enumerate(b.params):
                if p.requires_grad:
                    p.grad = gf[b.offsets[i]: b.offsets[i] + b.numels[i]].view(p.ds_shape)
        # parameters this unit's forward borrowed (register_external_parameter) are needed
        # by its backward too; their grads land in their owner's buffers
        for x in u.external:
            self._pre_backward(x)

    def _grad_ready(self, p):
        u = self._unit_of_param[id(p)]
        if u.reduced:
            # the unit's buffers were already reduced (reference stage3.py asserts the same:
            # a gradient computed twice in one backward, e.g. a parameter used both inside and
            # outside a reentrant-checkpointed region)
            raise RuntimeError(f"ZeRO-3: gradient of a parameter of unit {u.uid} ({type(u.module).__name__}) "
                               f"arrived after the unit was reduced; a parameter was used by two separate "
                               f"backward graph tasks")
        if not u.in_backward:
            # grad produced without the output hook firing (e.g. params used outside the
            # unit's forward): materialise the unit's grad buffers now and fold it in
            g_now = p.grad
            p.grad = None
            self._pre_backward(u)
            if g_now is not None:
                p.grad.add_(g_now)
        u.bw_ready += 1
        if u.bw_ready >= u.bw_expected:
            self._reduce_unit(u)

    def _reduce_unit(self, u: ZeroUnit):
        if u.reduced:
            return
        u.reduced = True
        u.in_backward = False
        for g, b in u.buckets:
            for p in b.params:
                p.grad = None
        if self.resident_grads and not self.is_gradient_accumulation_boundary:
            # keep accumulating into the unit's full buffers; reduce once at the boundary
            if u.active == 0:
                self._maybe_release(u, "b")
            return
        for (g, b), gf in zip(u.buckets, u.grad_fulls):
            src = gf
            if g.dtype == torch.float16:
                src.mul_(1.0 / self.dp_world)
            cast = None
            if self.fp32_reduce and src.dtype != torch.float32:
                # the fp32 staging copy of the unit gradient comes from (and returns to) the pool:
                # it is part of the planned transient memory, not a fresh allocation per unit
                cast = self._pool.get(src.numel(), torch.float32, src.device)
                cast.copy_(src)
                src = cast
            out_slice = g.shard_grad[b.shard_offset: b.shard_offset + b.chunk]
            direct = out_slice.dtype == src.dtype and not self._grads_nonzero
            out = out_slice if direct else self._pool.get(b.chunk, src.dtype, src.device)
            if self.use_reduce_scatter:
                work = comm.reduce_scatter_tensor(out, src, group=self.dp_group, async_op=True,
                                                  tag=f"zero3.reduce.u{u.uid}")
                done = None if direct else functools.partial(_accum, out_slice, out)
            else:
                work = comm.all_reduce(src, group=self.dp_group, async_op=True, tag=f"zero3.allreduce.u{u.uid}")
                mine = src[self.dp_rank * b.chunk: (self.dp_rank + 1) * b.chunk]
                done = functools.partial(_copy if direct else _accum, out_slice, mine)
            # buffers go back to the pool once the reduction has been waited for
            back = ([gf] if direct else [gf, out]) + ([cast] if cast is not None else [])
            fin = functools.partial(_finish_reduce, done, self._pool, back)
            self._reduced_this_pass = True
            self._queue_reduction(work, fin, b.numel, overlap=self.overlap_comm)
        u.grad_fulls = []
        if u.active == 0:
            self._maybe_release(u, "b")

    _grads_nonzero = False
    _reduced_this_pass = False

    def reduce_epilogue(self):
        if self.single:
            return
        for u in self._units:
            if u.in_backward and not u.reduced:
                self._reduce_unit(u)
        if self.resident_grads and self.is_gradient_accumulation_boundary:
            for u in self._units:  # accumulated in earlier micro-batches, unused in this one
                if u.grad_fulls and not u.reduced:
                    self._reduce_unit(u)
        self._drain_reductions()
        for u in self._units:
            u.reduced = False
            u.in_backward = False
            if u.active == 0 and u.status != ZeroParamStatus.NOT_AVAILABLE:
                self._maybe_release(u, "b")
        if self._reduced_this_pass:
            self._grads_nonzero = True
        self._reduced_this_pass = False
        if not self._trace_frozen and self._fwd_trace:
            self._trace_frozen = True
            self._compute_reuse()
        self._bwd_pos = 0

    overlapping_partition_gradients_reduce_epilogue = reduce_epilogue

    # ------------------------------------------------------------------ step
    def backward(self, loss, retain_graph=False):
        self.synchronize_step()
        self._bwd_pos = 0
        self.loss_scaler.backward(loss.float(), retain_graph=retain_graph)

    def _prescaled_by(self):
        return float(self.dp_world) if (self.groups and self.groups[0].dtype == torch.float16) else 1.0

    def _bucket_out(self, g, b):
        if self.param_nvme and g.shard_param is None:
            return self._pswap.staging(self._pkey[id(b)])
        return super()._bucket_out(g, b)

    def _after_bucket_update(self, g, b):
        if self.param_nvme and g.shard_param is None:
            self._pswap.swap_out(self._pkey[id(b)])
        if self._overlap_step and torch.cuda.current_stream() == self._step_stream:
            ev = torch.cuda.Event()
            ev.record(self._step_stream)
            self._bucket_events[self._bucket_key[id(b)]] = ev

    def _after_host_bucket_update(self, g, b, stream):
        if self._overlap_step and self._step_stream is not None:
            ev = torch.cuda.Event()
            ev.record(stream)
            self._bucket_events[self._bucket_key[id(b)]] = ev

    def state_dict(self):
        self.synchronize_step()
        return super().state_dict()

    def load_state_dict(self, *args, **kwargs):
        self.synchronize_step()
        return super().load_state_dict(*args, **kwargs)

    def param_shard_host(self, g) -> torch.Tensor:
        """This rank's low-precision shard of group g as a host tensor (checkpoints)."""
        if self.param_nvme and g.shard_param is None:
            out = torch.empty(g.shard_numel, dtype=g.dtype)
            self._pswap.synchronize_writes()
            for b in g.buckets:
                out[b.shard_offset: b.shard_offset + b.chunk].copy_(self._pswap.read(self._pkey[id(b)]))
            return out
        return g.shard_param.detach().cpu()

    def _low_precision_shard(self, g):
        if self.param_nvme and g.shard_param is None:
            return self.param_shard_host(g)
        return g.shard_param

    def load_param_shard(self, g, shard: torch.Tensor):
        if self.param_nvme and g.shard_param is None:
            for b in g.buckets:
                self._pswap.write(self._pkey[id(b)], shard[b.shard_offset: b.shard_offset + b.chunk])
            return
        g.shard_param.copy_(shard.to(g.shard_param.device))

    def _post_step(self):
        if self._pswap is not None:
            self._pswap.synchronize_writes()
        if self.single:
            return
        for u in self._units:  # retained gathered copies are stale after the update
            if not u.persistent and u.active == 0:
                self._release(u)
        for u in self._units:
            if u.persistent:
                self._release(u, force=True)
                self._fetch(u)
        for u in self._units:
            if u.persistent:
                self._wait(u)

    def zero_grad(self, set_to_none=True):
        self.synchronize_step()
        for g in self.groups:
            g.shard_grad.zero_()
        self._grads_nonzero = False
        for u in self._units:  # an overflow-skipped step drops resident micro-batch grads too
            for t in u.grad_fulls:
                self._pool.put(t)
            u.grad_fulls = []

    def _zero_stage(self):
        return 3

    # ------------------------------------------------------------------ memory knobs
    # Called between optimizer steps by a trainer that sizes HBM from measurement (bench.py:
    # a first step runs lean, the headroom it leaves is granted to retention / resident
    # gradients, and a later step that comes too close to the HBM limit gives them back).
    def set_max_live_parameters(self, numel: int):
        """stage3_max_live_parameters at run time; takes effect from the next gather (retained
        units above the new cap are dropped at the next step boundary, `_post_step`)."""
        self.max_live_parameters = max(0, int(numel))

    def set_resident_grads(self, enabled: bool):
        """Turn resident unit gradients on/off at an optimizer-step boundary.  The reduced
        shard gradient changes dtype with the mode under grad_accum_dtype "auto" (fp32 when
        GA > 1 micro-batch reductions land in it, param dtype with one reduction per step) and
        is re-allocated (zeroed: it is empty at a boundary)."""
        enabled = bool(enabled) and not self.single
        if enabled == self.resident_grads:
            return
        if any(u.grad_fulls for u in self._units) or self._grads_nonzero:
            raise RuntimeError("set_resident_grads() must be called between optimizer steps")
        self.resident_grads = enabled
        self.refresh_grad_dtype()

    def refresh_grad_dtype(self):
        """Re-allocate the (empty) reduced shard gradients when the accumulation mode (resident
        grads, gradient_accumulation_steps) changes the dtype they accumulate in."""
        if self.single:
            return
        for g in self.groups:
            gdt = self._grad_dtype(g)
            if g.shard_grad is not None and g.shard_grad.dtype != gdt:
                dev = g.shard_grad.device
                g.shard_grad = None
                g.shard_grad = torch.zeros(g.shard_numel, dtype=gdt, device=dev)
        self._pool.clear()

    def release_retained(self):
        """Drop every retained (non-persistent, idle) gathered unit and the pool's free buffers."""
        for u in self._units:
            if not u.persistent and u.active == 0:
                self._release(u)
        self._pool.clear()

    # ------------------------------------------------------------------ model state helpers
    def register_external_parameter(self, module, param):
        owner = self.unit_of(param)
        mu = self._unit_of_module.get(id(module))
        if owner is None or mu is None or owner is mu:
            return
        if owner not in mu.external:
            mu.external.append(owner)

    def write_back_params(self, params):
        """Copy edited full parameters (currently gathered) back into this rank's shard and
        fp32 master (zero.GatheredParameters(modifier_rank=...) exit path)."""
        want = {id(p) for p in params}
        for gi, g in enumerate(self.groups):
            if self.param_nvme and g.shard_param is None:
                shard = self.param_shard_host(g)
                g.shard_param = shard
                try:
                    self._write_back_group(gi, g, want)
                finally:
                    g.shard_param = None
                self.load_param_shard(g, shard)
                continue
            self._write_back_group(gi, g, want)

    def _write_back_group(self, gi, g, want):
        for bi, b in enumerate(g.buckets):
            nvme_master = None
            for i, p in enumerate(b.params):
                if id(p) not in want:
                    continue
                ov = b.chunk_overlap(self.dp_rank, i)
                if ov is None:
                    continue
                p0, c0, ln = ov
                lo = b.shard_offset + c0
                src = p.data.reshape(-1)[p0: p0 + ln]
                if g.shard_param[lo: lo + ln].data_ptr() != src.data_ptr():
                    g.shard_param[lo: lo + ln].copy_(src)
                if self.compact_master:
                    g.master[lo: lo + ln].zero_()
                elif self.nvme:  # fp32 master in the optimizer swap files
                    if nvme_master is None:
                        nvme_master = self._swapper.read((gi, bi), "master")
                    nvme_master[c0: c0 + ln].copy_(g.shard_param[lo: lo + ln].float().cpu())
                else:
                    g.master[lo: lo + ln].copy_(g.shard_param[lo: lo + ln].float().to(g.master.device))
            if nvme_master is not None:
                self._swapper.write((gi, bi), "master", nvme_master)

    def gathered_state_dict(self, module, prefix=""):
        """Full (consolidated) low-precision state dict; every rank participates."""
        out = {}
        for name, p in module.named_parameters(prefix=prefix.rstrip(".")):
            u = self.unit_of(p)
            if u is not None:
                was = u.status
                self.gather_units([u])
                out[name] = p.data.detach().clone().cpu()
                if was == ZeroParamStatus.NOT_AVAILABLE:
                    self._release(u)
            else:
                out[name] = p.detach().cpu()
        for name, bfr in module.named_buffers(prefix=prefix.rstrip(".")):
            out[name] = bfr.detach().cpu()
        return out


def _sole_owner(t) -> bool:
    """True when nothing but `t` (and its pool base) references its storage (the temporary
    storage handle of this query counts one)."""
    try:
        own = 2 if t._base is None else 3
        return torch._C._storage_Use_Count(t.untyped_storage()._cdata) <= own
    except Exception:  # noqa: BLE001 - private API; without it nothing is pooled
        return False


def _finish_reduce(done, pool, bufs):
    if done is not None:
        done()
    seen = set()
    for t in bufs:
        if id(t) not in seen:
            seen.add(id(t))
            pool.put(t)


def _accum(dst, src):
    dst.add_(src.to(dst.dtype))


def _copy(dst, src):
    dst.copy_(src)


FP16_DeepSpeedZeroOptimizer_Stage3 = DeepSpeedZeroOptimizer_Stage3
