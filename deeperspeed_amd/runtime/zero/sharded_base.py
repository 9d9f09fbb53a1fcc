"""Shared machinery of the flat-arena ZeRO optimizers (stages 0-3).

Reference parity (behaviour, not structure): loss scaling + overflow skip + grad-norm
clipping + inner step + fp16/bf16 copy-back of FP16_Optimizer (fp16/fused_optimizer.py:242-330)
and of the ZeRO wrappers (stage2.py:1366-1596, stage3.py:2742-2940); ZeRO checkpoint
state (stage2.py:1720-1880, stage3.py:3046-3160) including elastic re-partitioning when
the data-parallel world size changes; ZeRO-Offload of optimizer state (stage2.py:750-911).

MI355X design:
* Per group: one contiguous fp32 master shard, one contiguous gradient shard, Adam moments
  as flat tensors.  The step is one fused HIP launch per bucket chunk that reads the
  reduced gradient, updates master + moments and writes the bf16 model shard in the same
  pass (grad unscale and clip coefficient folded into a single scalar).
* Overflow + global grad norm come from one device-side sum-of-squares per shard plus a
  single all-reduce, then ONE host sync per step (reference: one per tensor).
* Offload ("cpu"): `states="all"` keeps master+moments in pinned host memory and steps with
  the native AVX-512 CPU Adam; `states="master"` (MI355X extension for 288 GB HBM) keeps
  the moments in HBM and streams the fp32 master through pinned staging buffers with
  H2D / kernel / D2H overlapped on separate HIP streams; `states="moments"` is the mirror
  image (moments on the host, master in HBM -- with compact_master only 6 B/param of HBM:
  the largest model one GPU trains, bounded by host memory at 8 B/param).
"""

from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ...ops import native
from ...utils import comm
from ...ops.adam.fused_adam import FusedAdam
from ...utils.logging import logger
from ..fp16.loss_scaler import DynamicLossScaler, LossScaler
from . import compact_master as cm
from .layout import FlatGroup, layout_signature, params_to_shard, shards_to_params
from .ref_layout import LAYOUT_VERSION, is_reference_layout, merge_reference_shards

# Host-moments groups: the Adam of the host-moments pieces runs on a stream of its own, the copies
# on two copy streams, beside the HBM groups.  Measured on the 20B N=1 step (profiles/r4q_notes.md,
# r4s_notes.md) against Adam after the HBM groups on the step stream (8,557-8,670 tok/s) and
# everything serial on the step stream (8,540-8,559): 8,868-8,972 tok/s; the write-back of m / v is
# torch's copy_ (a ROCclr blit kernel), which beat a 16-workgroup copy kernel (8,787 vs 8,720 tok/s,
# r4s_notes.md) and a hipMemcpy NoCU variant (the same blit path, r4p).  Those variants are gone.

OFFLOAD_SUBCHUNK = int(64 * 1024 * 1024)  # elements per staged piece (256 MB fp32)
# device staging slots of the states="moments" step (each holds one piece of m and v)
OFFLOAD_NBUF = 6  # 6 vs 3: +4 % at 30.3B (profiles/r4ag_notes.md)
CPU_STEP_PIECE = int(16 * 1024 * 1024)  # elements per CPU-Adam piece of the pipelined offload step


def _pipelined_offload() -> bool:
    """The pipelined D2H -> CPU Adam -> H2D offload step (GPU); the serial one on CPU-only hosts."""
    return torch.cuda.is_available()


class HostGradStream:
    """Reduced gradient pieces streamed to pinned host memory ahead of the CPU optimizer
    (reference: the async per-parameter D2H gradient copies of stage2.py:782-880).

    `get(k)` returns piece k on the host; before that it has issued the device-to-host
    copies of pieces k+1 .. k+depth on a dedicated HIP stream, so PCIe transfers of the next
    pieces overlap the CPU Adam of this one (and the H2D of the previous one's parameters).
    Gradients travel in their HBM dtype (bf16 shards: half the bytes of an fp32 copy); the
    CPU kernel widens them.  Slots are reused round-robin per dtype: piece k+depth takes
    the slot of a piece at least one position before k, which the CPU has finished."""

    def __init__(self, pieces, stream, depth=2):
        self.pieces = list(pieces)
        self.stream = stream
        self.depth = max(1, int(depth))
        self.slot_of = []
        seq, maxn = {}, {}
        for t in self.pieces:
            n = seq.get(t.dtype, 0)
            self.slot_of.append(n % (self.depth + 1))
            seq[t.dtype] = n + 1
            maxn[t.dtype] = max(maxn.get(t.dtype, 0), t.numel())
        self.slots = {dt: [torch.empty(n, dtype=dt, pin_memory=True) for _ in range(self.depth + 1)]
                      for dt, n in maxn.items()}
        self.ready = torch.cuda.Event()
        self.ready.record()  # gradients are final on the compute stream
        self.events = [None] * len(self.pieces)
        self.issued = 0

    def _issue(self, k):
        src = self.pieces[k]
        dst = self.slots[src.dtype][self.slot_of[k]][: src.numel()]
        with torch.cuda.stream(self.stream):
            if k == 0:
                self.stream.wait_event(self.ready)
            dst.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.events[k] = (ev, dst)

    def get(self, k):
        while self.issued < min(len(self.pieces), k + self.depth + 1):
            self._issue(self.issued)
            self.issued += 1
        ev, dst = self.events[k]
        ev.synchronize()
        self.events[k] = None
        return dst


def _is_mp_param(p):
    return bool(getattr(p, "model_parallel", False) or getattr(p, "tensor_model_parallel", False))


def _dist_ready():
    return dist.is_available() and dist.is_initialized()


class ShardedOptimizerBase:
    """Not an nn optimizer itself: wraps a client/basic torch optimizer (`init_optimizer`)."""

    def __init__(self, init_optimizer, dp_process_group=None, mpu=None, clip_grad=0.0, static_loss_scale=1.0,
                 dynamic_loss_scale=False, dynamic_loss_args=None, fp32_reduce=False, gradient_predivide_factor=1.0,
                 gradient_accumulation_steps=1, offload_optimizer=None, timers=None, verbose=False,
                 compact_master=False, sub_group_size=None):
        self.optimizer = init_optimizer
        # reference stage3.py:1332-1356: the optimizer steps over sub-groups of at most this
        # many elements (bounds the step's temporaries / host staging); here a sub-group is a
        # contiguous range of a group's shard, never larger than one bucket chunk
        self.sub_group_size = int(sub_group_size) if sub_group_size else 0
        self.compact_master = bool(compact_master)
        self.dp_group = dp_process_group
        self.mpu = mpu
        self.clip_grad = float(clip_grad or 0.0)
        self.fp32_reduce = bool(fp32_reduce)
        self.gradient_predivide_factor = float(gradient_predivide_factor or 1.0)
        self.gradient_accumulation_steps = int(gradient_accumulation_steps)
        self.timers = timers
        self.verbose = verbose
        # comm.world_size / rank: the real group's, or the N of an emulated world (bench.py
        # --emulate-world: shards, buckets and units of one rank of an N-rank job)
        self.dp_world = comm.world_size(dp_process_group)
        self.dp_rank = comm.rank(dp_process_group)
        self.mp_world = mpu.get_model_parallel_world_size() if mpu is not None else 1
        self.mp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
        if dynamic_loss_scale:
            self.loss_scaler = DynamicLossScaler(**(dynamic_loss_args or {}))
            self.dynamic_loss_scale = True
        else:
            self.loss_scaler = LossScaler(scale=static_loss_scale)
            self.dynamic_loss_scale = False
        self.overflow = False
        self.offload = offload_optimizer
        self.offload_states = (offload_optimizer or {}).get("states", "all") if offload_optimizer else None
        self.nvme = bool(offload_optimizer) and offload_optimizer.get("device") == "nvme"
        self._swapper = None
        self._mswap = None  # NVMe tier of offload states='moments' (_moment_tier)
        self._mswap_keys = {}
        self.fused = isinstance(init_optimizer, FusedAdam) or getattr(init_optimizer, "supports_flat_update", False)
        self.groups: List[FlatGroup] = []
        self.is_gradient_accumulation_boundary = True
        self._global_grad_norm = 0.0
        self._norm_buf = None
        self.device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
        self._copy_streams = None
        # host-moments groups (param groups with "host_moments": True, see _host_moments_step)
        self._host_stream = None
        self._host_staging = None
        self._host_d2h_done = None

    # ------------------------------------------------------------------ properties
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    @property
    def loss_scale(self):
        return self.loss_scaler.loss_scale

    @property
    def cur_scale(self):
        return self.loss_scaler.loss_scale

    def _get_loss_scale(self):
        return self.loss_scaler.loss_scale

    def _set_loss_scale(self, v):
        self.loss_scaler.cur_scale = v

    def get_global_grad_norm(self):
        return self._global_grad_norm

    # ------------------------------------------------------------------ setup helpers
    def _host_moment_group(self, g) -> bool:
        """Param groups marked `"host_moments": True` keep their Adam moments in pinned host
        memory while the rest of the optimizer state stays in HBM (MI355X extension: frees
        8 B / parameter of HBM for the groups a trainer names -- bench.py gives it to the GPT-NeoX
        LM head and last layers, whose update has the most slack before the next forward reads
        them).  Needs the fused Adam and a GPU; the step streams the moments through HBM in
        pieces on copy engines (_host_moments_step)."""
        return bool(self.optimizer.param_groups[g.group_index].get("host_moments", False)) and self.fused \
            and torch.cuda.is_available() and self.offload is None

    def _moment_tier(self, g) -> str:
        """Where group g's Adam moments live under offload_optimizer states='moments': the param
        group's "moments_device" ("cpu" = pinned host, "nvme" = an aio-swapped file, "gpu" = HBM),
        default "cpu".  Three tiers let a single GPU train a model whose moments exceed any one of
        HBM headroom, the host-memory budget and the disk (bench.py --offload moments sizes them)."""
        if not (self.offload is not None and self.offload_states == "moments"):
            return "gpu"
        t = str(self.optimizer.param_groups[g.group_index].get("moments_device", "cpu")).lower()
        if t not in ("cpu", "nvme", "gpu", "hbm"):
            raise ValueError(f"moments_device must be cpu, nvme or gpu, got {t!r}")
        return "gpu" if t == "hbm" else t

    def _split_groups(self):
        """Split each inner param group into (dtype, model-parallel) flat groups."""
        from .layout import split_param_group
        out = []
        # registration order of every param group (reference-layout checkpoint import)
        self._orig_group_params = [list(pg["params"]) for pg in self.optimizer.param_groups]
        for gi, pg in enumerate(self.optimizer.param_groups):
            for si, (dt, mp, plist) in enumerate(split_param_group(pg["params"], _is_mp_param)):
                out.append(FlatGroup(group_index=gi, sub_index=si, dtype=dt, model_parallel=mp, params=plist))
        return out

    def _alloc_master_and_state(self, init_shard_fn):
        """Create master shards from `init_shard_fn(group) -> fp32 tensor [S]` on the
        right device, rebind inner optimizer param groups to the masters."""
        host = self.offload is not None and self.offload.get("device") in ("cpu", "nvme")
        pin = bool(self.offload and self.offload.get("pin_memory", True)) and torch.cuda.is_available()
        moments_only = self.offload is not None and self.offload_states == "moments"
        if moments_only and (self.offload.get("device") != "cpu" or not self.fused or not torch.cuda.is_available()):
            raise ValueError("offload_optimizer states='moments' needs device 'cpu', the fused Adam optimizer and a GPU")
        host = host and not moments_only  # the master stays in HBM
        if self.compact_master:
            if (self.offload is not None and not moments_only) or not self.fused:
                raise ValueError("compact_master needs the fused Adam optimizer and no optimizer offload "
                                 "(or offload_optimizer states='moments')")
            for g in self.groups:
                if g.dtype != torch.bfloat16 or g.shard_param is None:
                    raise ValueError("compact_master needs bf16 model parameters")
        if self.nvme:
            self._setup_nvme(init_shard_fn)
            return
        for g in self.groups:
            if self.compact_master:
                # the bf16 shard already equals the master's high half: residual starts at 0
                g.master = torch.zeros(g.shard_numel, dtype=torch.int16, device=g.shard_param.device)
                continue
            m = init_shard_fn(g).float()
            if host:
                hm = native.pinned_zeros(g.shard_numel, torch.float32) if pin else \
                    torch.empty(g.shard_numel, dtype=torch.float32)
                hm.copy_(m)
                m = hm
            g.master = m
            g.master.requires_grad_(False)
        # rebind optimizer groups: params -> masters of their flat groups
        for gi, pg in enumerate(self.optimizer.param_groups):
            pg["params"] = [g.master for g in self.groups if g.group_index == gi]
        self.optimizer.state.clear()
        # moments: allocated up-front so memory is visible and offload placement is explicit
        if self.fused or self.offload is not None:
            for g in self.groups:
                st = self.optimizer.state[g.master]
                st["step"] = 0
                tier = self._moment_tier(g) if moments_only else None
                if tier == "nvme":
                    self._register_nvme_moments(g)
                    st["exp_avg"] = torch.zeros(0, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros(0, dtype=torch.float32)
                    continue
                on_host = (host and self.offload_states == "all") or (moments_only and tier == "cpu") or \
                    self._host_moment_group(g)
                kw = dict(dtype=torch.float32, pin_memory=on_host and (pin or moments_only or
                                                                       self._host_moment_group(g)))
                if on_host:
                    if kw["pin_memory"]:  # exact-size page-locked memory (native.pinned_zeros)
                        st["exp_avg"] = native.pinned_zeros(g.shard_numel, torch.float32)
                        st["exp_avg_sq"] = native.pinned_zeros(g.shard_numel, torch.float32)
                    else:
                        st["exp_avg"] = torch.zeros(g.shard_numel, **kw)
                        st["exp_avg_sq"] = torch.zeros(g.shard_numel, **kw)
                else:
                    st["exp_avg"] = torch.zeros(g.shard_numel, dtype=torch.float32, device=self.device)
                    st["exp_avg_sq"] = torch.zeros(g.shard_numel, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ NVMe tier of the moments
    def _register_nvme_moments(self, g):
        """Zero-initialised exp_avg / exp_avg_sq files for every bucket of group g."""
        import os
        from ..swap_tensor.optimizer_utils import PipelinedOptimizerSwapper
        if self._mswap is None:
            path = self.offload.get("nvme_path") or "/tmp/deeperspeed_amd_nvme"
            folder = os.path.join(path, f"zero_stage_{self._zero_stage()}_moments",
                                  f"rank{self.dp_rank}_mp{self.mp_rank}")
            self._mswap = PipelinedOptimizerSwapper(folder, names=("exp_avg", "exp_avg_sq"),
                                                    aio_config=self.offload.get("aio") or {})
        gi = self.groups.index(g)
        for bi, b in enumerate(g.buckets):
            if b.chunk > 0:
                self._mswap.register((gi, bi), {}, numel=b.chunk)
                self._mswap_keys[(gi, bi)] = b

    def _nvme_moments_group(self, gi, name) -> torch.Tensor:
        g = self.groups[gi]
        parts = [self._mswap.read((gi, bi), name) for bi, b in enumerate(g.buckets) if b.chunk > 0]
        return torch.cat(parts) if parts else torch.zeros(0)

    def _nvme_moments_write(self, gi, name, value: torch.Tensor):
        g = self.groups[gi]
        value = value.reshape(-1).float().cpu()
        for bi, b in enumerate(g.buckets):
            if b.chunk > 0:
                self._mswap.write((gi, bi), name, value[b.shard_offset: b.shard_offset + b.chunk])

    # ------------------------------------------------------------------ NVMe (ZeRO-Infinity)
    def _setup_nvme(self, init_shard_fn):
        """fp32 master + Adam moments live on NVMe, one file per (group, bucket, tensor); the
        step streams them through pinned buffers (runtime/swap_tensor/optimizer_utils.py)."""
        import os
        from ..swap_tensor.optimizer_utils import PipelinedOptimizerSwapper, log_swap_config
        path = self.offload.get("nvme_path") or "/tmp/deeperspeed_amd_nvme"
        folder = os.path.join(path, f"zero_stage_{self._zero_stage()}", f"rank{self.dp_rank}_mp{self.mp_rank}")
        aio = self.offload.get("aio") or {}
        self._swapper = PipelinedOptimizerSwapper(folder, aio_config=aio)
        log_swap_config(folder, aio)
        for gi, g in enumerate(self.groups):
            m = init_shard_fn(g).float()
            for bi, b in enumerate(g.buckets):
                lo, hi = b.shard_offset, b.shard_offset + b.chunk
                self._swapper.register((gi, bi), {"master": m[lo:hi].detach().cpu()})
            del m
            g.master = torch.zeros(0, dtype=torch.float32)  # placeholder key for the inner optimizer
        for gi, pg in enumerate(self.optimizer.param_groups):
            pg["params"] = [g.master for g in self.groups if g.group_index == gi]
        self.optimizer.state.clear()
        for g in self.groups:
            self.optimizer.state[g.master] = {"step": 0, "exp_avg": torch.zeros(0), "exp_avg_sq": torch.zeros(0)}

    def _nvme_read_group(self, gi, name) -> torch.Tensor:
        g = self.groups[gi]
        return torch.cat([self._swapper.read((gi, bi), name) for bi in range(len(g.buckets))]) if g.buckets \
            else torch.zeros(0)

    def _nvme_write_group(self, gi, name, value: torch.Tensor):
        g = self.groups[gi]
        value = value.reshape(-1).float().cpu()
        for bi, b in enumerate(g.buckets):
            self._swapper.write((gi, bi), name, value[b.shard_offset: b.shard_offset + b.chunk])

    def _offload_nvme_step(self, grad_scale, grp_steps):
        from ...ops.adam.cpu_adam import cpu_adam_update_flat
        adamw = bool(getattr(self.optimizer, "adam_w_mode", getattr(self.optimizer, "adamw_mode", True)))
        keys = [(gi, bi) for gi, g in enumerate(self.groups) for bi in range(len(g.buckets))]
        stream = None
        if _pipelined_offload() and any(g.shard_grad.is_cuda for g in self.groups):
            stream = HostGradStream([self.groups[gi].shard_grad[self.groups[gi].buckets[bi].shard_offset:
                                                                 self.groups[gi].buckets[bi].shard_offset +
                                                                 self.groups[gi].buckets[bi].chunk]
                                     for gi, bi in keys], self._streams()[0])
        order = {k: i for i, k in enumerate(keys)}

        def update(key, t):
            gi, bi = key
            g = self.groups[gi]
            b = g.buckets[bi]
            lo, hi = b.shard_offset, b.shard_offset + b.chunk
            grad_host = stream.get(order[key]) if stream is not None else g.shard_grad[lo:hi]
            cpu_adam_update_flat(t["master"], grad_host, t["exp_avg"], t["exp_avg_sq"], self._inner_group(g),
                                 grp_steps[id(g)], grad_scale, adamw, out_device=self._bucket_out(g, b))
            self._after_bucket_update(g, b)

        self._swapper.update(keys, update)

    def _step_pieces(self, b):
        """(lo, hi) shard ranges of bucket b, each at most sub_group_size elements."""
        lo, hi = b.shard_offset, b.shard_offset + b.chunk
        step = self.sub_group_size if 0 < self.sub_group_size < b.chunk else b.chunk
        step = max(step, 64)  # keep pieces vector-aligned and non-degenerate
        return [(s, min(s + step, hi)) for s in range(lo, hi, step)] or [(lo, hi)]

    def _inner_group(self, g: FlatGroup):
        return self.optimizer.param_groups[g.group_index]

    # ------------------------------------------------------------------ in-flight reductions
    # ProcessGroupNCCL keeps an async collective's tensors alive until its work is waited
    # for, so an unbounded queue of gradient reductions would hold every bucket/unit gradient
    # buffer of the backward at once (the whole model's gradients).  The queue is bounded by
    # element count: once more than `max_inflight_numel` elements are in flight the oldest
    # reductions are completed.  work.wait() on RCCL only makes the compute stream wait for
    # the collective's stream (no host block), so draining early costs no CPU run-ahead.
    max_inflight_numel = 0  # 0 = two of the largest reductions

    def _queue_reduction(self, work, fin, numel=0, overlap=True):
        if not overlap:
            if work is not None:
                work.wait()
            if fin is not None:
                fin()
            return
        pend = self.__dict__.setdefault("_pending", [])
        pend.append((work, fin, int(numel)))
        self._inflight = getattr(self, "_inflight", 0) + int(numel)
        self._inflight_peak = max(getattr(self, "_inflight_peak", 0), int(numel))
        cap = self.max_inflight_numel or 2 * self._inflight_peak
        while len(pend) > 1 and self._inflight > cap:
            self._complete_oldest()

    def _complete_oldest(self):
        work, fin, numel = self._pending.pop(0)
        self._inflight -= numel
        if work is not None:
            work.wait()
        if fin is not None:
            fin()

    def _drain_reductions(self):
        while getattr(self, "_pending", None):
            self._complete_oldest()
        self._inflight = 0

    # ------------------------------------------------------------------ norm / overflow
    def _shard_grads_for_norm(self):
        """Yield (tensor, include) pairs whose sum of squares forms this rank's share."""
        for g in self.groups:
            if g.shard_grad is None:
                continue
            # replicated (non model-parallel) params are counted on mp rank 0 only
            include = g.model_parallel or self.mp_rank == 0
            yield g.shard_grad, include

    def _grads_are_sharded(self):
        return True

    def _compute_norm_sq(self) -> torch.Tensor:
        if self._norm_buf is None:
            self._norm_buf = torch.zeros(1, dtype=torch.float32, device=self.device)
        buf = self._norm_buf
        buf.zero_()
        for t, include in self._shard_grads_for_norm():
            if include:
                native.sumsq_accumulate(t, buf)
        if _dist_ready():
            if self._grads_are_sharded() and self.dp_world > 1:
                comm.all_reduce(buf, group=self.dp_group, tag="zero.norm")
            if self.mp_world > 1:
                dist.all_reduce(buf, group=self.mpu.get_model_parallel_group())
        return buf

    def _grad_divisor(self):
        """Total factor the summed gradients must be divided by (loss scale * averaging)."""
        return self.loss_scale * self._avg_divisor()

    def _avg_divisor(self):
        return float(self.dp_world) / self._prescaled_by()

    def _prescaled_by(self):
        return 1.0

    # ------------------------------------------------------------------ step
    def _unscale_and_clip_coef(self, total_sq: float):
        div = self._grad_divisor()
        norm = math.sqrt(total_sq) / div if total_sq >= 0 else float("nan")
        self._global_grad_norm = norm
        coef = 1.0
        if self.clip_grad > 0 and norm > self.clip_grad:
            coef = self.clip_grad / (norm + 1e-6)
        return coef / div, norm

    def _check_overflow_and_scale(self):
        total = float(self._compute_norm_sq().item())  # the one host sync per step
        overflow = not math.isfinite(total)
        self.overflow = overflow
        if self.dynamic_loss_scale or overflow:
            prev = self.loss_scale
            self.loss_scaler.update_scale(overflow)
            if overflow:
                logger.info(f"[deepspeed] OVERFLOW! Skipping step. Attempted loss scale: {prev}, reducing to "
                            f"{self.loss_scale}")
        return overflow, total

    def step(self, closure=None):
        if comm.DEBUG:
            comm.verify_collective_order(self.dp_group)
        if self.timers is not None:
            self.timers("optimizer_step").start()
        overflow, total = self._check_overflow_and_scale()
        if overflow:
            self.zero_grad()
            if self.timers is not None:
                self.timers("optimizer_step").stop()
            return
        grad_scale, _ = self._unscale_and_clip_coef(total)
        self._inner_step(grad_scale)
        self._post_step()
        self.zero_grad()
        if self.timers is not None:
            self.timers("optimizer_step").stop()

    def _bucket_out(self, g: FlatGroup, b):
        """Low-precision destination (view) of bucket b's shard chunk after the update."""
        return g.shard_param[b.shard_offset: b.shard_offset + b.chunk]

    def _after_bucket_update(self, g: FlatGroup, b):
        pass

    def _post_step(self):
        pass

    def _inner_step(self, grad_scale: float):
        if self.offload is not None:
            return self._offload_step(grad_scale)
        if self.fused:
            for g in self.groups:
                st = self.optimizer.state_for(g.master) if isinstance(self.optimizer, FusedAdam) else \
                    self.optimizer.state[g.master]
                st["step"] = st.get("step", 0) + 1
            host_groups = [g for g in self.groups if self._host_moment_group(g)]
            if host_groups:  # copy pipeline + kernels beside the HBM groups
                self._host_moments_step(host_groups, grad_scale)
            for g in self.groups:
                if self._host_moment_group(g):
                    continue
                grp = self._inner_group(g)
                for b in g.buckets:
                    out = self._bucket_out(g, b)
                    for lo, hi in self._step_pieces(b):
                        o = None if out is None else out[lo - b.shard_offset: hi - b.shard_offset]
                        self.optimizer.update_flat(grp, g.master, g.master, g.shard_grad, out=o,
                                                   grad_scale=grad_scale, lo=lo, hi=hi)
                    self._after_bucket_update(g, b)
            if host_groups:  # the step's end (and the gradient zeroing after it) follows their kernels
                torch.cuda.current_stream().wait_stream(self._host_stream)
            return
        # generic torch optimizer over the fp32 master shards
        for g in self.groups:
            gr = g.shard_grad.float() if g.shard_grad.dtype != torch.float32 else g.shard_grad.clone()
            gr.mul_(grad_scale)
            g.master.grad = gr
        self.optimizer.step()
        for g in self.groups:
            g.master.grad = None
            for b in g.buckets:
                out = self._bucket_out(g, b)
                if out is not None and out.data_ptr() != g.master.data_ptr():
                    native.scale_copy_(g.master[b.shard_offset: b.shard_offset + b.chunk], out)
                self._after_bucket_update(g, b)

    HOST_PIECE = int(16 * 1024 * 1024)  # elements of m / v staged per piece (64 MB each in fp32)

    def _host_moments_step(self, groups, grad_scale):
        """Adam for the host-moments groups: per piece, H2D of m / v into one of three persistent
        HBM staging slots (copy stream), the fused Adam kernel on a stream of its own, D2H of m / v
        (second copy stream).  Nothing waits on the host: the current stream (the overlapped
        step's side stream, or the compute stream) waits for the kernels at the end, the next
        step's H2D waits for this step's D2H, and checkpoints wait for it (host_moments_sync).
        Each bucket's update event is recorded for the forward pre-hooks (overlap_step)."""
        h2d, d2h = self._streams()
        if self._host_stream is None:
            self._host_stream = self._new_stream()
        hs, cur = self._host_stream, torch.cuda.current_stream()
        piece = min(self.HOST_PIECE, max(b.chunk for g in groups for b in g.buckets))
        if self._host_staging is None or self._host_staging[0][0].numel() < piece:
            self._host_staging = [(torch.empty(piece, dtype=torch.float32, device=self.device),
                                   torch.empty(piece, dtype=torch.float32, device=self.device)) for _ in range(3)]
        stages = self._host_staging
        start = torch.cuda.Event()
        start.record(cur)  # gradients are final
        hs.wait_event(start)
        h2d.wait_event(start)
        if self._host_d2h_done is not None:  # the previous step's moments are home
            h2d.wait_event(self._host_d2h_done)
        free_ev = list(getattr(self, "_host_free_ev", [None] * 3))
        adamw = bool(getattr(self.optimizer, "adam_w_mode", True))
        k = 0
        for g in groups:
            grp = self._inner_group(g)
            b1, b2 = grp["betas"]
            st = self.optimizer.state_for(g.master) if isinstance(self.optimizer, FusedAdam) else \
                self.optimizer.state[g.master]
            for b in g.buckets:
                out_full = self._bucket_out(g, b)
                for s in range(0, b.chunk, piece):
                    e = min(s + piece, b.chunk)
                    lo, hi, n = b.shard_offset + s, b.shard_offset + e, e - s
                    i = k % 3
                    k += 1
                    m_dev, v_dev = stages[i][0][:n], stages[i][1][:n]
                    with torch.cuda.stream(h2d):
                        if free_ev[i] is not None:
                            h2d.wait_event(free_ev[i])
                        m_dev.copy_(st["exp_avg"][lo:hi], non_blocking=True)
                        v_dev.copy_(st["exp_avg_sq"][lo:hi], non_blocking=True)
                        ev_in = torch.cuda.Event()
                        ev_in.record(h2d)
                    hs.wait_event(ev_in)
                    o = None if out_full is None else out_full[s:e]
                    with torch.cuda.stream(hs):
                        if self.compact_master:
                            native.adam_compact_(o, g.master[lo:hi], g.shard_grad[lo:hi], m_dev, v_dev, grp["lr"],
                                                 b1, b2, grp["eps"], grp["weight_decay"], st["step"],
                                                 grp.get("bias_correction", True), grad_scale, adamw)
                        else:
                            native.adam_flat_(g.master[lo:hi], g.shard_grad[lo:hi], m_dev, v_dev, o, grp["lr"], b1,
                                              b2, grp["eps"], grp["weight_decay"], st["step"],
                                              grp.get("bias_correction", True), grad_scale, adamw)
                        ev_done = torch.cuda.Event()
                        ev_done.record(hs)
                    with torch.cuda.stream(d2h):
                        d2h.wait_event(ev_done)
                        st["exp_avg"][lo:hi].copy_(m_dev, non_blocking=True)
                        st["exp_avg_sq"][lo:hi].copy_(v_dev, non_blocking=True)
                        ev_free = torch.cuda.Event()
                        ev_free.record(d2h)
                    free_ev[i] = ev_free
                self._after_host_bucket_update(g, b, hs)
        self._host_free_ev = free_ev
        done = torch.cuda.Event()
        done.record(d2h)
        self._host_d2h_done = done

    def _after_host_bucket_update(self, g, b, stream):
        """Bucket-update hook for a host-moments bucket updated on `stream` (stage 3 records the
        overlap_step event there)."""

    def host_moments_sync(self):
        """Block the host until the last step's host moments are written back (checkpoints)."""
        if self._host_d2h_done is not None:
            self._host_d2h_done.synchronize()

    # ------------------------------------------------------------------ offload step
    def _streams(self):
        if self._copy_streams is None and torch.cuda.is_available():
            self._copy_streams = (self._new_stream(), self._new_stream())
        return self._copy_streams

    def _new_stream(self):
        from ..overlap_step import dedicated_stream, new_stream
        if self.offload is not None:
            # an offloaded step IS the critical path (nothing computes beside it): its copy
            # streams get hardware queues of their own, or a copy stream's waits can stall the
            # compute stream's Adam kernels behind them in a shared queue (profiles/r4ag_notes.md)
            return dedicated_stream(self.device)
        return new_stream(self.device)

    def _offload_step(self, grad_scale: float):
        grp_steps = {}
        for g in self.groups:
            st = self.optimizer.state[g.master]
            st["step"] = st.get("step", 0) + 1
            grp_steps[id(g)] = st["step"]
        if self.nvme:
            return self._offload_nvme_step(grad_scale, grp_steps)
        if self.offload_states == "master" and torch.cuda.is_available():
            return self._offload_master_step(grad_scale, grp_steps)
        if self.offload_states == "moments":
            return self._offload_moments_step(grad_scale, grp_steps)
        return self._offload_all_step(grad_scale, grp_steps)

    def _offload_master_step(self, grad_scale, grp_steps):
        """fp32 master in pinned host memory, moments + grads in HBM.  Pipeline per piece:
        H2D master (stream A) -> fused Adam (compute) -> D2H master (stream B)."""
        h2d, d2h = self._streams()
        cur = torch.cuda.current_stream()
        nbuf = 3
        piece = min(OFFLOAD_SUBCHUNK, max(b.chunk for g in self.groups for b in g.buckets))
        stages = [torch.empty(piece, dtype=torch.float32, device=self.device) for _ in range(nbuf)]
        free_ev = [None] * nbuf
        k = 0
        for g in self.groups:
            grp = self._inner_group(g)
            st = self.optimizer.state[g.master]
            for b in g.buckets:
                out_full = self._bucket_out(g, b)
                for s in range(0, b.chunk, piece):
                    e = min(s + piece, b.chunk)
                    lo, hi, n = b.shard_offset + s, b.shard_offset + e, e - s
                    i = k % nbuf
                    k += 1
                    buf = stages[i][:n]
                    with torch.cuda.stream(h2d):
                        if free_ev[i] is not None:
                            h2d.wait_event(free_ev[i])
                        buf.copy_(g.master[lo:hi], non_blocking=True)
                        ev_in = torch.cuda.Event()
                        ev_in.record(h2d)
                    cur.wait_event(ev_in)
                    b1, b2 = grp["betas"]
                    native.adam_flat_(buf, g.shard_grad[lo:hi], st["exp_avg"][lo:hi], st["exp_avg_sq"][lo:hi],
                                      out_full[s:e] if out_full is not None else None, grp["lr"], b1, b2, grp["eps"],
                                      grp["weight_decay"], grp_steps[id(g)], grp.get("bias_correction", True),
                                      grad_scale, bool(getattr(self.optimizer, "adam_w_mode", True)))
                    ev_done = torch.cuda.Event()
                    ev_done.record(cur)
                    with torch.cuda.stream(d2h):
                        d2h.wait_event(ev_done)
                        g.master[lo:hi].copy_(buf, non_blocking=True)
                        ev_free = torch.cuda.Event()
                        ev_free.record(d2h)
                    free_ev[i] = ev_free
                self._after_bucket_update(g, b)
        # host master must be final before the next step reads it (and before checkpoints)
        d2h.synchronize()
        del stages

    def _moments_kernel(self, g, grp, o, lo, hi, m, v, step, grad_scale, adamw):
        b1, b2 = grp["betas"]
        if self.compact_master:
            native.adam_compact_(o, g.master[lo:hi], g.shard_grad[lo:hi], m, v, grp["lr"], b1, b2, grp["eps"],
                                 grp["weight_decay"], step, grp.get("bias_correction", True), grad_scale, adamw)
        else:
            native.adam_flat_(g.master[lo:hi], g.shard_grad[lo:hi], m, v, o, grp["lr"], b1, b2, grp["eps"],
                              grp["weight_decay"], step, grp.get("bias_correction", True), grad_scale, adamw)

    def _offload_moments_step(self, grad_scale, grp_steps):
        """Adam moments off-HBM, master (compact or fp32) and gradients in HBM.  Three tiers, per
        param group (_moment_tier): HBM-resident moments update in place; pinned-host moments
        stream per piece: H2D of m, v (stream A) -> fused Adam on the compute stream -> D2H of m, v
        (stream B), three device staging slots keeping both copy engines and the kernel busy;
        NVMe moments (_nvme_moments_step) are read / written by the aio engine on the host while
        their H2D / Adam / D2H run on a stream of their own, beside the host tier."""
        h2d, d2h = self._streams()
        cur = torch.cuda.current_stream()
        adamw = bool(getattr(self.optimizer, "adam_w_mode", True))
        tiers = {id(g): self._moment_tier(g) for g in self.groups}
        for g in self.groups:  # HBM tier: no copies
            if tiers[id(g)] != "gpu":
                continue
            grp, st = self._inner_group(g), self.optimizer.state[g.master]
            for b in g.buckets:
                out_full = self._bucket_out(g, b)
                lo, hi = b.shard_offset, b.shard_offset + b.chunk
                self._moments_kernel(g, grp, out_full, lo, hi, st["exp_avg"][lo:hi], st["exp_avg_sq"][lo:hi],
                                     grp_steps[id(g)], grad_scale, adamw)
                self._after_bucket_update(g, b)
        host_groups = [g for g in self.groups if tiers[id(g)] == "cpu"]
        nvme_groups = [g for g in self.groups if tiers[id(g)] == "nvme"]
        if not host_groups:
            if nvme_groups:
                self._nvme_moments_step(nvme_groups, grad_scale, grp_steps, adamw)
            return
        nbuf = OFFLOAD_NBUF
        piece = min(OFFLOAD_SUBCHUNK // 2, max(b.chunk for g in host_groups for b in g.buckets))
        stages = [(torch.empty(piece, dtype=torch.float32, device=self.device),
                   torch.empty(piece, dtype=torch.float32, device=self.device)) for _ in range(nbuf)]
        free_ev = [None] * nbuf
        start = torch.cuda.Event()
        start.record(cur)  # gradients are final
        k = 0
        for g in host_groups:
            grp = self._inner_group(g)
            b1, b2 = grp["betas"]
            st = self.optimizer.state[g.master]
            for b in g.buckets:
                out_full = self._bucket_out(g, b)
                for s in range(0, b.chunk, piece):
                    e = min(s + piece, b.chunk)
                    lo, hi, n = b.shard_offset + s, b.shard_offset + e, e - s
                    i = k % nbuf
                    k += 1
                    m_dev, v_dev = stages[i][0][:n], stages[i][1][:n]
                    with torch.cuda.stream(h2d):
                        h2d.wait_event(start)
                        if free_ev[i] is not None:
                            h2d.wait_event(free_ev[i])
                        m_dev.copy_(st["exp_avg"][lo:hi], non_blocking=True)
                        v_dev.copy_(st["exp_avg_sq"][lo:hi], non_blocking=True)
                        ev_in = torch.cuda.Event()
                        ev_in.record(h2d)
                    cur.wait_event(ev_in)
                    o = None if out_full is None else out_full[s:e]
                    if self.compact_master:
                        native.adam_compact_(o, g.master[lo:hi], g.shard_grad[lo:hi], m_dev, v_dev, grp["lr"], b1, b2,
                                             grp["eps"], grp["weight_decay"], grp_steps[id(g)],
                                             grp.get("bias_correction", True), grad_scale, adamw)
                    else:
                        native.adam_flat_(g.master[lo:hi], g.shard_grad[lo:hi], m_dev, v_dev, o, grp["lr"], b1, b2,
                                          grp["eps"], grp["weight_decay"], grp_steps[id(g)],
                                          grp.get("bias_correction", True), grad_scale, adamw)
                    ev_done = torch.cuda.Event()
                    ev_done.record(cur)
                    with torch.cuda.stream(d2h):
                        d2h.wait_event(ev_done)
                        st["exp_avg"][lo:hi].copy_(m_dev, non_blocking=True)
                        st["exp_avg_sq"][lo:hi].copy_(v_dev, non_blocking=True)
                        ev_free = torch.cuda.Event()
                        ev_free.record(d2h)
                    free_ev[i] = ev_free
                self._after_bucket_update(g, b)
        if nvme_groups:  # its host loop runs while the GPU works through the host tier above
            self._nvme_moments_step(nvme_groups, grad_scale, grp_steps, adamw)
        # host moments final before a checkpoint or the next step reads them; staging buffers
        # are released only after the copies that use them
        cur.wait_stream(d2h)
        d2h.synchronize()
        del stages

    NVME_PIECE = int(32 * 1024 * 1024)  # elements of m / v per H2D / Adam / D2H piece of the NVMe tier

    def _nvme_moments_step(self, groups, grad_scale, grp_steps, adamw):
        """NVMe tier of the moments.  The aio engine reads bucket k+1's m / v files into pinned
        buffers and writes bucket k-1's back while bucket k runs H2D -> fused Adam -> D2H on a
        stream of its own (PipelinedOptimizerSwapper); the host waits for that stream once per
        bucket before its buffers are written back."""
        cur = torch.cuda.current_stream()
        if getattr(self, "_nvme_stream", None) is None:
            self._nvme_stream = self._new_stream()
        ns = self._nvme_stream
        start = torch.cuda.Event()
        start.record(cur)  # gradients are final
        ns.wait_event(start)
        keys = [k for k, b in self._mswap_keys.items() if self.groups[k[0]] in groups]
        piece = min(self.NVME_PIECE, max(self._mswap_keys[k].chunk for k in keys))
        m_dev = torch.empty(piece, dtype=torch.float32, device=self.device)
        v_dev = torch.empty(piece, dtype=torch.float32, device=self.device)

        t0, done_n = time.time(), [0]

        def update(key, t):
            gi, bi = key
            g, b = self.groups[gi], self._mswap_keys[key]
            done_n[0] += 1
            if done_n[0] % 64 == 0:
                logger.debug(f"NVMe moments tier: {done_n[0]}/{len(keys)} buckets, {time.time() - t0:.1f}s, "
                            f"{self._mswap.bytes_read / 2**30:.1f} GiB read")
            grp = self._inner_group(g)
            out_full = self._bucket_out(g, b)
            with torch.cuda.stream(ns):
                for s0 in range(0, b.chunk, piece):
                    e0 = min(s0 + piece, b.chunk)
                    n, lo, hi = e0 - s0, b.shard_offset + s0, b.shard_offset + e0
                    m, v = m_dev[:n], v_dev[:n]
                    m.copy_(t["exp_avg"][s0:e0], non_blocking=True)
                    v.copy_(t["exp_avg_sq"][s0:e0], non_blocking=True)
                    self._moments_kernel(g, grp, None if out_full is None else out_full[s0:e0], lo, hi, m, v,
                                         grp_steps[id(g)], grad_scale, adamw)
                    t["exp_avg"][s0:e0].copy_(m, non_blocking=True)
                    t["exp_avg_sq"][s0:e0].copy_(v, non_blocking=True)
                done = torch.cuda.Event()
                done.record(ns)
            done.synchronize()  # m / v are home in the pinned buffers: the swapper writes them next
            self._after_bucket_update(g, b)

        self._mswap.update(keys, update)
        cur.wait_stream(ns)
        del m_dev, v_dev

    def _offload_all_step(self, grad_scale, grp_steps):
        """Reference ZeRO-Offload: master + moments on host, native CPU Adam.  Pipelined over
        pieces of at most CPU_STEP_PIECE elements: D2H of the next gradient pieces (copy
        stream) and H2D of the previous piece's bf16 parameters (double-buffered pinned
        staging) run while the CPU updates the current piece."""
        from ...ops.adam.cpu_adam import cpu_adam_update_flat
        adamw = bool(getattr(self.optimizer, "adam_w_mode", True))
        work = []  # (group, bucket, lo, hi, last piece of the bucket)
        for g in self.groups:
            for b in g.buckets:
                lo0, hi0 = b.shard_offset, b.shard_offset + b.chunk
                cuts = list(range(lo0, hi0, CPU_STEP_PIECE)) or [lo0]
                for i, lo in enumerate(cuts):
                    work.append((g, b, lo, min(lo + CPU_STEP_PIECE, hi0), i == len(cuts) - 1))
        stream = None
        if _pipelined_offload() and any(g.shard_grad.is_cuda for g in self.groups):
            stream = HostGradStream([g.shard_grad[lo:hi] for g, _, lo, hi, _ in work], self._streams()[0])
        bucket_out = None
        for k, (g, b, lo, hi, last) in enumerate(work):
            grad_host = stream.get(k) if stream is not None else g.shard_grad[lo:hi]
            st = self.optimizer.state[g.master]
            if lo == b.shard_offset:  # once per bucket (NVMe params: acquires one staging buffer)
                bucket_out = self._bucket_out(g, b)
            out = None if bucket_out is None else bucket_out[lo - b.shard_offset: hi - b.shard_offset]
            cpu_adam_update_flat(g.master[lo:hi], grad_host, st["exp_avg"][lo:hi], st["exp_avg_sq"][lo:hi],
                                 self._inner_group(g), grp_steps[id(g)], grad_scale, adamw, out_device=out)
            if last:
                self._after_bucket_update(g, b)

    # ------------------------------------------------------------------ grads
    def zero_grad(self, set_to_none=True):
        for g in self.groups:
            if g.shard_grad is not None:
                g.shard_grad.zero_()

    # ------------------------------------------------------------------ checkpoint
    def _zero_stage(self):
        return 0

    def state_dict(self):
        self.host_moments_sync()
        base = self.optimizer.state_dict()
        if self.nvme:  # moments live on NVMe: materialise them for the checkpoint
            for gi in range(len(self.groups)):
                st = base.get("state", {}).get(gi)
                if st is not None:
                    st["exp_avg"] = self._nvme_read_group(gi, "exp_avg")
                    st["exp_avg_sq"] = self._nvme_read_group(gi, "exp_avg_sq")
        if self._mswap is not None:  # NVMe tier of offload states='moments'
            for gi, g in enumerate(self.groups):
                st = base.get("state", {}).get(gi)
                if st is not None and self._moment_tier(g) == "nvme":
                    st["exp_avg"] = self._nvme_moments_group(gi, "exp_avg")
                    st["exp_avg_sq"] = self._nvme_moments_group(gi, "exp_avg_sq")
        # move state tensors to cpu (checkpoint files are host tensors)
        for k, v in base.get("state", {}).items():
            for kk, vv in list(v.items()):
                if torch.is_tensor(vv):
                    v[kk] = vv.detach().cpu()
        sd = {
            "loss_scaler": self.loss_scaler.state_dict(),
            "dynamic_loss_scale": self.dynamic_loss_scale,
            "overflow": self.overflow,
            "base_optimizer_state": base,
            "zero_stage": self._zero_stage(),
            "partition_count": self.dp_world,
            "layout": layout_signature(self.groups),
            "dsa_layout_version": LAYOUT_VERSION,
            "fp32_groups_key": self._fp32_key(),
            self._fp32_key(): [self.master_fp32(g) for g in self.groups],
        }
        return sd

    def _fp32_key(self):
        # NOT the reference's key names (single_partition_of_fp32_groups / fp32_flat_groups):
        # these shards are interleaved per bucket, and reference tools must fail on them
        # rather than silently mis-read them (ref_layout.py)
        return "dsa_flat_fp32_shards"

    def load_state_dict(self, state_dict_list, load_optimizer_states=True, load_from_fp32_weights=True):
        self.host_moments_sync()  # no write-back of the previous step may land after the load
        if isinstance(state_dict_list, dict):
            state_dict_list = [state_dict_list]
        sd0 = state_dict_list[0]
        ls = sd0.get("loss_scaler")
        if isinstance(ls, dict):
            self.loss_scaler.load_state_dict(ls)
        elif ls is not None and hasattr(ls, "cur_scale"):  # reference checkpoints pickle the scaler object
            self.loss_scaler.load_state_dict({k: getattr(ls, k) for k in
                                              ("cur_scale", "cur_iter", "last_overflow_iter", "cur_hysteresis")
                                              if hasattr(ls, k)})
        self.dynamic_loss_scale = sd0.get("dynamic_loss_scale", self.dynamic_loss_scale)
        self.overflow = sd0.get("overflow", False)
        key = sd0.get("fp32_groups_key", self._fp32_key())
        lw, lr = self._layout_world_rank()
        if sd0.get("zero_stage", 0) == 0:
            state_dict_list = state_dict_list[:1]  # unsharded: every rank saved the same full state
        same_layout = (len(state_dict_list) == lw and sd0.get("layout") == layout_signature(self.groups))
        if is_reference_layout(sd0):
            masters, moments = self._import_reference_layout(state_dict_list)
        elif same_layout:
            mine = state_dict_list[lr]
            masters = mine[key]
            moments = mine["base_optimizer_state"]
        else:
            masters, moments = self._elastic_merge(state_dict_list, key)
        if load_from_fp32_weights:
            for gi, (g, m) in enumerate(zip(self.groups, masters)):
                if self.nvme:
                    self._nvme_write_group(gi, "master", m)
                    continue
                if self.compact_master:
                    cm.encode_into(m, g.shard_param, g.master)
                else:
                    g.master.copy_(m.to(g.master.device))
            self._refresh_params_from_master()
        else:
            # reference stage2.py:1877-1880 (_restore_from_fp16_weights): the low-precision
            # weights just loaded with the module become the masters
            self._masters_from_low_precision()
        if load_optimizer_states:
            self._load_moments(moments)

    def _layout_world_rank(self):
        """(world, rank) of the shard layout (unsharded stage 0 uses a world of 1)."""
        return self.dp_world, self.dp_rank

    def _elastic_merge(self, sds, key):
        """Re-partition masters and moments saved under a different DP world size."""
        _, my_rank = self._layout_world_rank()
        masters, moments_state = [], {}
        sig_list = sds[0]["layout"]
        old_base = [sd["base_optimizer_state"] for sd in sds]
        for gi, g in enumerate(self.groups):
            sig = sig_list[gi]
            full = shards_to_params([sd[key][gi] for sd in sds], sig)
            masters.append(params_to_shard(full, g, my_rank, torch.float32))
            st_new = {}
            for name in ("exp_avg", "exp_avg_sq"):
                olds = [ob["state"].get(gi, {}).get(name) for ob in old_base]
                if all(o is not None for o in olds):
                    st_new[name] = params_to_shard(shards_to_params(olds, sig), g, my_rank, torch.float32)
            step = old_base[0]["state"].get(gi, {}).get("step", 0)
            st_new["step"] = step
            moments_state[gi] = st_new
        return masters, {"state": moments_state, "param_groups": old_base[0]["param_groups"]}

    def _import_reference_layout(self, sds):
        """Masters + moments of a reference (contiguous per-group) ZeRO checkpoint, re-partitioned
        into this rank's shards of the current layout (any saved world size)."""
        numels = [[p.ds_numel if hasattr(p, "ds_numel") else p.numel() for p in plist]
                  for plist in self._orig_group_params]
        ref_masters, ref_moments = merge_reference_shards(sds, numels)
        _, my_rank = self._layout_world_rank()
        masters, state = [], {}
        for gi, g in enumerate(self.groups):
            pos = {id(p): j for j, p in enumerate(self._orig_group_params[g.group_index])}
            mine = [pos[id(p)] for p in g.params]
            masters.append(params_to_shard({i: ref_masters[g.group_index][j] for i, j in enumerate(mine)}, g,
                                           my_rank, torch.float32))
            mom = ref_moments[g.group_index]
            st = {"step": mom.get("step", 0)}
            for k in ("exp_avg", "exp_avg_sq"):
                if k in mom:
                    st[k] = params_to_shard({i: mom[k][j] for i, j in enumerate(mine)}, g, my_rank, torch.float32)
            state[gi] = st
        logger.info(f"imported a reference-layout ZeRO-{sds[0].get('zero_stage')} checkpoint saved by "
                    f"{len(sds)} ranks into {self._layout_world_rank()[0]} ranks")
        return masters, {"state": state, "param_groups": []}

    def _load_moments(self, base_sd):
        # param groups hyper-params (lr etc.) restored; state tensors copied in place
        saved_groups = base_sd.get("param_groups", [])
        for pg, spg in zip(self.optimizer.param_groups, saved_groups):
            for k, v in spg.items():
                if k != "params":
                    pg[k] = v
        states = base_sd.get("state", {})
        for gi, g in enumerate(self.groups):
            s = states.get(gi)
            if s is None:
                continue
            st = self.optimizer.state[g.master]
            for k, v in s.items():
                if self.nvme and torch.is_tensor(v) and k in ("exp_avg", "exp_avg_sq"):
                    self._nvme_write_group(gi, k, v)
                elif (self._mswap is not None and torch.is_tensor(v) and k in ("exp_avg", "exp_avg_sq")
                      and self._moment_tier(g) == "nvme"):
                    self._nvme_moments_write(gi, k, v)
                elif torch.is_tensor(v) and k in st and torch.is_tensor(st[k]) and st[k].numel() == v.numel():
                    st[k].copy_(v.to(st[k].device))
                elif torch.is_tensor(v):
                    st[k] = v.to(g.master.device if not (self.offload and self.offload_states == "all")
                                 else "cpu").clone()
                else:
                    st[k] = v

    def _low_precision_shard(self, g: FlatGroup) -> torch.Tensor:
        return g.shard_param

    def _masters_from_low_precision(self):
        """fp32 masters <- this rank's low-precision parameter shards (compact: the bf16 shard
        is the master's high half, the residual restarts at zero)."""
        for gi, g in enumerate(self.groups):
            src = self._low_precision_shard(g)
            if src is None:
                continue
            if self.compact_master:
                g.master.zero_()
            elif self.nvme:
                self._nvme_write_group(gi, "master", src.float())
            elif g.master.data_ptr() != src.data_ptr():
                g.master.copy_(src.float().to(g.master.device))

    def master_fp32(self, g: FlatGroup) -> torch.Tensor:
        """This rank's fp32 master shard of group g as a host tensor (checkpoints, tests)."""
        if self.nvme:
            return self._nvme_read_group(self.groups.index(g), "master")
        if self.compact_master:
            return cm.decode_chunked(g.shard_param, g.master, torch.empty(g.shard_numel, dtype=torch.float32))
        return g.master.detach().cpu()

    def _refresh_params_from_master(self):
        """Copy master -> low-precision shard/params after a fp32 restore."""
        for g in self.groups:
            for b in g.buckets:
                out = self._bucket_out(g, b)
                if self.nvme:
                    if out is not None:
                        out.copy_(self._swapper.read((self.groups.index(g), g.buckets.index(b)), "master")
                                  .to(out.device, out.dtype))
                elif self.compact_master:
                    pass  # the bf16 shard is the master's high half already
                elif out is not None and out.data_ptr() != g.master.data_ptr():
                    out.copy_(g.master[b.shard_offset: b.shard_offset + b.chunk].to(out.device))
                self._after_bucket_update(g, b)
        self._post_step()
