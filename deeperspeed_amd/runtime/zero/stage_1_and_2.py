"""Data-parallel mixed precision and ZeRO stages 1 / 2 on the flat-arena layout.

Reference parity: FP16_Optimizer (fp16/fused_optimizer.py), ZeRO-1
(zero/stage1.py: optimizer-state partitioning, reduce-scatter, all-gather after step) and
ZeRO-2 (zero/stage2.py: gradient partitioning with IPG buckets reduced during backward,
`overlap_comm`, ZeRO-Offload).  Behaviour differences by design (MI355X / RCCL):

* Parameters of a group live in one arena; all-gather after the step writes each bucket
  in place with ONE `all_gather_into_tensor` (reference: `num_shards` pieces,
  stage2.py:1480-1516).
* Gradient reduction is ONE `reduce_scatter_tensor` per bucket (reference ZeRO-2 issues N
  `dist.reduce` calls per bucket, stage2.py:695-745), launched from post-accumulate-grad
  hooks as buckets fill during backward, in a rank-consistent order, on RCCL's stream.
* Stage 0 (plain DP + mixed precision) uses the same code with an unsharded layout and
  an in-place all-reduce per bucket; grads are views into a flat arena (no copies).
* fp32 communication (`fp32_allreduce`, DeeperSpeed bf16 default) upcasts bucket-by-bucket
  and *keeps* the fp32 result (the reference discards it, stage2.py:731-745).
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ...utils import comm
from ...utils.logging import logger
from .layout import ALIGN, FlatGroup, build_size_buckets
from .sharded_base import ShardedOptimizerBase, _dist_ready


class _BucketState:
    __slots__ = ("expected", "ready", "launched", "buffer", "order")

    def __init__(self, expected, order):
        self.expected = expected
        self.ready = 0
        self.launched = False
        self.buffer = None
        self.order = order


class DeepSpeedZeroOptimizer(ShardedOptimizerBase):
    def __init__(self, init_optimizer, stage=1, dp_process_group=None, mpu=None, clip_grad=0.0,
                 static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None, reduce_bucket_size=int(5e8),
                 allgather_bucket_size=int(5e8), overlap_comm=True, reduce_scatter=True, fp32_reduce=False,
                 gradient_predivide_factor=1.0, gradient_accumulation_steps=1, offload_optimizer=None, timers=None,
                 postscale_gradients=True, verbose=False, compact_master=False, resident_grads=False,
                 sub_group_size=None, prebind_window=2):
        super().__init__(init_optimizer, dp_process_group=dp_process_group, mpu=mpu, clip_grad=clip_grad,
                         static_loss_scale=static_loss_scale, dynamic_loss_scale=dynamic_loss_scale,
                         dynamic_loss_args=dynamic_loss_args, fp32_reduce=fp32_reduce,
                         gradient_predivide_factor=gradient_predivide_factor,
                         gradient_accumulation_steps=gradient_accumulation_steps,
                         offload_optimizer=offload_optimizer, timers=timers, verbose=verbose,
                         compact_master=compact_master, sub_group_size=sub_group_size)
        assert stage in (0, 1, 2)
        self.stage = stage
        self.sharded = stage >= 1
        self.layout_world = self.dp_world if self.sharded else 1
        # overlap_comm=False (reference stage2.py:680-686): each bucket's reduction is waited
        # for where it is issued instead of at the end of backward
        self.overlap_comm = True if overlap_comm is None else bool(overlap_comm)
        # reduce_scatter=False (reference stage2.py:687): all-reduce each bucket, keep the chunk
        self.use_reduce_scatter = bool(reduce_scatter)
        # MI355X extension for ZeRO-2: hold a full gradient arena (like stage 1) so micro-batch
        # gradients accumulate in place and every bucket is reduce-scattered once per optimizer
        # step; on 288 GB parts this usually fits next to the full bf16 parameter arena
        self.resident = stage == 2 and bool(resident_grads)
        # ZeRO-2 without a resident arena: the next `prebind_window` buckets (backward order)
        # get pooled buffers bound as p.grad before their gradients arrive, so autograd
        # accumulates straight into the bucket instead of a copy per parameter
        self.prebind_window = max(1, int(prebind_window))
        self.reduce_bucket_size = max(int(reduce_bucket_size), ALIGN * max(1, self.dp_world))
        self.max_inflight_numel = 2 * self.reduce_bucket_size
        self.groups = self._split_groups()
        for g in self.groups:
            build_size_buckets(g, self.layout_world, self.reduce_bucket_size)
        self._build_arenas()
        self._build_grad_storage()
        self._alloc_master_and_state(self._initial_master)
        self._register_hooks()
        self._pending = []  # (work, finisher)
        self._buf_pool: Dict[torch.dtype, List[torch.Tensor]] = {}
        self._reset_bucket_states()
        if verbose:
            n = sum(p.numel() for g in self.groups for p in g.params)
            logger.info(f"ZeRO stage {stage}: {len(self.groups)} flat groups, "
                        f"{sum(len(g.buckets) for g in self.groups)} buckets, {n / 1e6:.1f}M params, "
                        f"dp_world={self.dp_world}")

    # ------------------------------------------------------------------ layout
    def _build_arenas(self):
        for g in self.groups:
            dev = g.params[0].device
            g.arena = torch.zeros(g.arena_numel, dtype=g.dtype, device=dev)
            for b in g.buckets:
                for p, off, n in zip(b.params, b.offsets, b.numels):
                    view = g.arena[b.arena_offset + off: b.arena_offset + off + n]
                    view.copy_(p.data.reshape(-1))
                    p.data = view.view(p.shape)
        self._pos = {}
        for g in self.groups:
            for b in g.buckets:
                for i, p in enumerate(b.params):
                    self._pos[p] = (g, b, i)
        if not self.sharded:
            for g in self.groups:
                g.shard_param = g.arena  # unsharded: the "shard" is the whole arena
        else:
            for g in self.groups:
                g.shard_param = torch.empty(g.shard_numel, dtype=g.dtype, device=g.arena.device)
                for b in g.buckets:
                    c0 = b.arena_offset + self.dp_rank * b.chunk
                    g.shard_param[b.shard_offset: b.shard_offset + b.chunk].copy_(g.arena[c0: c0 + b.chunk])

    def _initial_master(self, g: FlatGroup):
        if g.dtype == torch.float32 and not self.sharded and self.offload is None:
            return g.arena  # fp32 model, stage 0: the params ARE the master
        return g.shard_param.float()

    def _alloc_master_and_state(self, init_shard_fn):
        super()._alloc_master_and_state(init_shard_fn)
        for g in self.groups:
            if g.master.data_ptr() == g.arena.data_ptr() if g.arena is not None else False:
                g.shard_param = None  # update in place, nothing to copy back

    def _bucket_out(self, g, b):
        if g.shard_param is None:
            return None
        return g.shard_param[b.shard_offset: b.shard_offset + b.chunk]

    def _grad_dtype(self, g):
        if self.fp32_reduce or g.dtype == torch.float32:
            return torch.float32
        if self._bucketed() and self.gradient_accumulation_steps > 1:
            return torch.float32  # GA reductions accumulate in the shard
        return g.dtype

    def _bucketed(self):
        """ZeRO-2 proper: gradients live in pooled bucket buffers during backward only."""
        return self.stage == 2 and not self.resident

    def _build_grad_storage(self):
        for g in self.groups:
            dev = g.arena.device
            if not self._bucketed():
                g.grad_arena = torch.zeros(g.arena_numel, dtype=g.dtype, device=dev)
                for b in g.buckets:
                    for p, off, n in zip(b.params, b.offsets, b.numels):
                        p.grad = g.grad_arena[b.arena_offset + off: b.arena_offset + off + n].view(p.shape)
            gdt = self._grad_dtype(g)
            if self.stage == 0 and gdt == g.dtype:
                g.shard_grad = g.grad_arena  # all-reduce in place
            else:
                g.shard_grad = torch.zeros(g.shard_numel, dtype=gdt, device=dev)

    def _register_hooks(self):
        self._hook_handles = []
        for g in self.groups:
            for p in g.params:
                self._hook_handles.append(p.register_post_accumulate_grad_hook(self._grad_ready))
        # rank-consistent launch order: by position of the bucket's first param in the global
        # reverse-registration order (~ backward order), ties by group.
        all_params = [p for g in self.groups for p in g.params]
        rev_pos = {id(p): i for i, p in enumerate(reversed(all_params))}
        keys = []
        for gi, g in enumerate(self.groups):
            for b in g.buckets:
                keys.append((min(rev_pos[id(p)] for p in b.params), gi, b.index, g, b))
        keys.sort(key=lambda t: (t[0], t[1], t[2]))
        self._launch_seq = [(g, b) for _, _, _, g, b in keys]

    def _reset_bucket_states(self):
        self._bstate = {}
        for i, (g, b) in enumerate(self._launch_seq):
            exp = sum(1 for p in b.params if p.requires_grad)
            self._bstate[id(b)] = _BucketState(exp, i)
        self._next_launch = 0

    # ------------------------------------------------------------------ backward hooks
    def _hooks_active(self):
        return self._bucketed() or self.is_gradient_accumulation_boundary

    def _acquire_buffer(self, g, b):
        pool = self._buf_pool.setdefault(g.dtype, [])
        size = max(bb.numel for gg in self.groups for bb in gg.buckets if gg.dtype == g.dtype)
        buf = pool.pop() if pool else torch.empty(size, dtype=g.dtype, device=g.arena.device)
        view = buf[: b.numel]
        view.zero_()
        return buf, view

    def _prebind(self, k):
        """Bind bucket k (launch order) to a pooled buffer: its params' .grad become views."""
        if k >= len(self._launch_seq):
            return
        g, b = self._launch_seq[k]
        st = self._bstate[id(b)]
        if st.buffer is not None or st.launched:
            return
        st.buffer = self._acquire_buffer(g, b)
        for i, p in enumerate(b.params):
            if p.requires_grad and p.grad is None:
                off = b.offsets[i]
                p.grad = st.buffer[1][off: off + b.numels[i]].view(p.shape)

    def _grad_ready(self, p):
        if not self._hooks_active():
            return
        g, b, i = self._pos[p]
        st = self._bstate[id(b)]
        if self._bucketed():
            if st.buffer is None:
                st.buffer = self._acquire_buffer(g, b)
            off = b.offsets[i]
            dst = st.buffer[1][off: off + b.numels[i]]
            if p.grad is not None and p.grad.data_ptr() != dst.data_ptr():
                dst.copy_(p.grad.reshape(-1))  # arrived before its bucket was pre-bound
                p.grad = None
        st.ready += 1
        if st.ready >= st.expected:
            self._launch_ready_in_order()

    def _launch_ready_in_order(self, force=False):
        while self._next_launch < len(self._launch_seq):
            g, b = self._launch_seq[self._next_launch]
            st = self._bstate[id(b)]
            if not force and st.ready < st.expected:
                return
            self._launch_bucket(g, b, st)
            self._next_launch += 1

    def _launch_bucket(self, g: FlatGroup, b, st: _BucketState):
        st.launched = True
        world = self.dp_world
        if self._bucketed():
            if st.buffer is None:  # no grads at all arrived (unused params)
                st.buffer = self._acquire_buffer(g, b)
            src = st.buffer[1]
            for p in b.params:
                p.grad = None  # the buffer goes to the collective and back to the pool
            self._prebind(st.order + self.prebind_window)
        else:
            src = g.grad_arena[b.arena_offset: b.arena_offset + b.numel]
        dst_full = g.shard_grad
        red_dtype = torch.float32 if self.fp32_reduce else g.dtype
        if g.dtype == torch.float16:
            src.mul_(1.0 / world)  # fp16: pre-divide to stay in range
        if red_dtype != src.dtype:
            src = src.float()
        if self.stage == 0:
            if dst_full is g.grad_arena:
                target = src
            else:
                target = dst_full[b.shard_offset: b.shard_offset + b.numel]
                target.copy_(src)
            work = comm.all_reduce(target, group=self.dp_group, async_op=True, tag="zero.allreduce") if (_dist_ready() and world > 1) \
                else None
            self._queue(work, None, b.numel)
            return
        out_slice = dst_full[b.shard_offset: b.shard_offset + b.chunk]
        accumulate = self._bucketed() and self.gradient_accumulation_steps > 1
        staged = accumulate or out_slice.dtype != src.dtype or not self.use_reduce_scatter
        out = out_slice
        if _dist_ready() and world > 1 and self.use_reduce_scatter:
            if staged:  # reduce-scatter into a staging buffer only where finish() must convert / add
                out = torch.empty(b.chunk, dtype=src.dtype, device=src.device)
            work = comm.reduce_scatter_tensor(out, src, group=self.dp_group, async_op=True, tag="zero.reduce")
        elif _dist_ready() and world > 1:
            work = comm.all_reduce(src, group=self.dp_group, async_op=True, tag="zero.allreduce")
            out = src[self.dp_rank * b.chunk: (self.dp_rank + 1) * b.chunk]
        else:
            if not staged:
                out.copy_(src[: b.chunk])
            else:  # one rank: finish() reads the bucket itself (no staging copy)
                out = src[: b.chunk]
            work = None

        def finish(out=out, out_slice=out_slice, accumulate=accumulate, st=st, g=g):
            if out is not out_slice:
                if accumulate:
                    # bf16 micro-batch gradient into the fp32 shard: one fused cast-accumulate pass
                    from ...ops import native
                    native.scale_copy_(out, out_slice, 1.0, accumulate=True)
                else:
                    out_slice.copy_(out)
            if st.buffer is not None:
                self._buf_pool.setdefault(g.dtype, []).append(st.buffer[0])
                st.buffer = None

        self._queue(work, finish, b.numel)

    def _queue(self, work, fin, numel=0):
        self._queue_reduction(work, fin, numel, overlap=self.overlap_comm)

    def reduce_epilogue(self):
        """Flush all buckets and complete their reductions (end of backward)."""
        if not self._hooks_active():
            return
        self._launch_ready_in_order(force=True)
        self._drain_reductions()
        self._reset_bucket_states()

    # reference method names
    overlapping_partition_gradients_reduce_epilogue = reduce_epilogue

    def reduce_scatter_gradients(self, postscale_gradients=True, gradient_predivide_factor=1.0,
                                 gradient_average=True):
        self.reduce_epilogue()

    # ------------------------------------------------------------------ forward/backward API
    def backward(self, loss, retain_graph=False):
        if self._bucketed():
            for k in range(self.prebind_window):
                self._prebind(k)
        self.loss_scaler.backward(loss.float(), retain_graph=retain_graph)

    def _grads_are_sharded(self):
        return self.sharded

    def _prescaled_by(self):
        return float(self.dp_world) if (self.groups and self.groups[0].dtype == torch.float16) else 1.0

    def _after_bucket_update(self, g, b):
        if not self.sharded:
            return
        full = g.arena[b.arena_offset: b.arena_offset + b.numel]
        chunk = g.shard_param[b.shard_offset: b.shard_offset + b.chunk]
        if _dist_ready() and self.dp_world > 1:
            w = comm.all_gather_into_tensor(full, chunk, group=self.dp_group, async_op=True, tag="zero.gather")
            self._ag_works.append(w)
        else:
            full[: b.chunk].copy_(chunk)

    def _inner_step(self, grad_scale):
        self._ag_works = []
        super()._inner_step(grad_scale)

    def _post_step(self):
        for w in getattr(self, "_ag_works", []):
            w.wait()
        self._ag_works = []

    def _refresh_params_from_master(self):
        self._ag_works = []
        super()._refresh_params_from_master()

    def refresh_from_params(self):
        """Re-derive shards and fp32 masters from the (just loaded) model parameters."""
        if self.sharded:
            for g in self.groups:
                for b in g.buckets:
                    c0 = b.arena_offset + self.dp_rank * b.chunk
                    g.shard_param[b.shard_offset: b.shard_offset + b.chunk].copy_(g.arena[c0: c0 + b.chunk])
        super()._masters_from_low_precision()

    def _low_precision_shard(self, g):
        return g.shard_param if g.shard_param is not None else g.arena

    def _masters_from_low_precision(self):
        self.refresh_from_params()  # arena (loaded module weights) -> shard -> master

    def zero_grad(self, set_to_none=True):
        for g in self.groups:
            if g.grad_arena is not None:
                g.grad_arena.zero_()
            if g.shard_grad is not None and g.shard_grad is not g.grad_arena:
                g.shard_grad.zero_()

    def _zero_stage(self):
        return self.stage

    def _layout_world_rank(self):
        return (self.dp_world, self.dp_rank) if self.sharded else (1, 0)

    def _fp32_key(self):
        return super()._fp32_key() if self.sharded else "fp32_groups_flat"


# reference class names
FP16_DeepSpeedZeroOptimizer = DeepSpeedZeroOptimizer


class FP16_DeepSpeedZeroOptimizer_Stage1(DeepSpeedZeroOptimizer):
    def __init__(self, init_optimizer, **kw):
        kw.setdefault("stage", 1)
        super().__init__(init_optimizer, **kw)


class FP16_Optimizer(DeepSpeedZeroOptimizer):
    """Non-ZeRO mixed precision (stage 0 of the flat-arena optimizer)."""

    def __init__(self, init_optimizer, **kw):
        kw["stage"] = 0
        super().__init__(init_optimizer, **kw)
