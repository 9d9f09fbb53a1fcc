"""Mixed-precision wrapper with one fp32 master per parameter (no flattening).

Reference parity: deepspeed/runtime/fp16/unfused_optimizer.py:1-407 (`FP16_UnfusedOptimizer`),
used for optimizers whose math is per-tensor (LAMB's trust ratio): flattening the model into
one arena would merge the per-layer norms.  bf16/fp16 gradients are unscaled and clipped
straight into the fp32 master grads (one fused pass per tensor), the inner optimizer runs on
the masters and the low-precision params are refreshed from them.  The data-parallel
all-reduce of the model gradients is done by the engine before `step` (engine.py
buffered_allreduce_fallback), exactly like the reference.
"""

import math

import torch
import torch.distributed as dist

from ...utils.logging import logger
from ..utils import CheckOverflow, get_grad_norm, grad_norm_sq_tensor
from .loss_scaler import DynamicLossScaler, LossScaler


# bf16 / static-scale steps without a host read of the gradient norm
SYNC_FREE_STEP = True


class FP16_UnfusedOptimizer:
    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None,
                 verbose=True, mpu=None, clip_grad=0.0, fused_lamb_legacy=False, overlap_step=False, module=None,
                 overlap_bucket_numel=8_000_000):
        self.optimizer = init_optimizer
        self.mpu = mpu
        self.clip_grad = float(clip_grad or 0.0)
        self.fused_lamb_legacy = fused_lamb_legacy
        self.fp16_groups, self.fp32_groups = [], []
        for group in self.optimizer.param_groups:
            lp = list(group["params"])
            masters = []
            for p in lp:
                m = p.detach().clone().float()
                m.requires_grad_(False)
                masters.append(m)
            self.fp16_groups.append(lp)
            self.fp32_groups.append(masters)
            group["params"] = masters
        if dynamic_loss_scale:
            self.loss_scaler = DynamicLossScaler(**(dynamic_loss_args or {}))
            self.dynamic_loss_scale = True
        else:
            self.loss_scaler = LossScaler(scale=static_loss_scale)
            self.dynamic_loss_scale = False
        self.overflow = False
        self.overflow_checker = CheckOverflow(self.fp16_groups, mpu=mpu)
        self._global_grad_norm = 0.0
        self._overlap = None
        self._persistent_zeroed = False  # set by an overlapped step that zeroed them itself
        self._dev_skipped = None  # device count of sync-free steps skipped as non-finite
        self._skips_seen = 0
        if overlap_step:
            self._setup_overlap(module, overlap_bucket_numel, verbose)
        if verbose:
            logger.info(f"FP16_UnfusedOptimizer: {sum(len(g) for g in self.fp16_groups)} params with fp32 masters")

    # ----------------------------------------------------------------- properties
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

    def reconcile_skipped_steps(self) -> int:
        """Sync-free steps skip a non-finite update inside the kernels, unseen by the host.  This
        reads the device-side count (one host sync: call it at print / checkpoint boundaries),
        rolls the per-parameter step counters back by the newly skipped steps so later bias
        corrections are right again, and returns that number for the engine's skipped-step
        accounting.  Steps taken between a skip and this call used a bias correction one step
        ahead (documented drift; the LR schedule is not rolled back either)."""
        if self._dev_skipped is None:
            return 0
        n = int(self._dev_skipped.item()) - self._skips_seen
        if n <= 0:
            return 0
        self._skips_seen += n
        for st in self.optimizer.state.values():
            if "step" in st:
                st["step"] = max(0, st["step"] - n)
        logger.warning(f"[deepspeed] {n} sync-free LAMB step(s) had a non-finite gradient norm and were skipped "
                       f"on the device; optimizer step counters rolled back")
        return n

    def get_global_grad_norm(self):
        if torch.is_tensor(self._global_grad_norm):  # sync-free step: read on demand only
            self._global_grad_norm = float(self._global_grad_norm)
        return self._global_grad_norm

    def _sync_free(self, params):
        """Static loss scale 1 (bf16) with the fused multi-tensor LAMB: the unscale x clip factor
        is formed on the device and a non-finite gradient norm makes the kernels skip the update
        (LambArgs.scale_ptr), so the step needs no host read and the host keeps queueing the next
        forward.  The host-side overflow flag then stays False (the skipped-step count and the LR
        schedule are not rolled back on the -- for bf16 diverged -- non-finite step)."""
        return (SYNC_FREE_STEP and not self.dynamic_loss_scale and self.loss_scale == 1.0
                and getattr(self.optimizer, "supports_device_scale", False) and params
                and all(p.is_cuda for p in params))

    def _device_coef(self, params):
        sq = grad_norm_sq_tensor(params, mpu=self.mpu)
        norm = sq.sqrt()
        self._global_grad_norm = norm
        coef = torch.ones_like(norm)
        if self.clip_grad > 0:
            coef = torch.where(norm > self.clip_grad, self.clip_grad / (norm + 1e-6), coef)
        return torch.where(torch.isfinite(sq), coef, torch.full_like(coef, float("nan")))

    # ----------------------------------------------------------------- overlapped step
    def _setup_overlap(self, module, bucket_numel, verbose):
        """zero_optimization.overlap_step on the per-tensor path (runtime/overlap_step.py): the
        fused LAMB of a step runs on a side stream in forward-ordered buckets while the next
        forward starts; each module waits only for its own bucket."""
        params = [p for g in self.fp16_groups for p in g]
        ok = (module is not None and getattr(self.optimizer, "supports_fused_lp_step", False)
              and hasattr(self.optimizer, "step_subset") and torch.cuda.is_available() and params
              and all(p.is_cuda for p in params))
        if not ok:
            if verbose:
                logger.info("overlap_step: needs a fused low-precision optimizer (FusedLamb) on the GPU; "
                            "running the step serially")
            return
        from ..overlap_step import OverlapStep, forward_order_buckets
        where = [(gi, i) for gi, g in enumerate(self.fp16_groups) for i in range(len(g))]
        flat_buckets = forward_order_buckets(module, params, bucket_numel)
        # per bucket: {group index: [param index within the group]}
        self._overlap_buckets = []
        for idxs in flat_buckets:
            by_group = {}
            for k in idxs:
                gi, i = where[k]
                by_group.setdefault(gi, []).append(i)
            self._overlap_buckets.append(by_group)
        self._overlap = OverlapStep(module, params, flat_buckets, params[0].device)
        if verbose:
            logger.info(f"overlap_step: {len(flat_buckets)} forward-ordered optimizer buckets on a side stream")

    def synchronize_step(self):
        """Order the current stream after an overlapped step (checkpointing, state access)."""
        if self._overlap is not None:
            self._overlap.synchronize()

    def _overlapped_fused_step(self, coef_t):
        ov = self._overlap
        with ov.launch():
            for key, by_group in enumerate(self._overlap_buckets):
                persistent = []
                for gi, idxs in by_group.items():
                    lp = self.fp16_groups[gi]
                    grads = [lp[i].grad for i in idxs]
                    self.optimizer.step_subset(gi, idxs, grads, [lp[i].data for i in idxs], coef_t)
                    persistent += [g for i, g in zip(idxs, grads)
                                   if g is not None and getattr(lp[i], "_dsa_persistent_grad", False)]
                # persistent (HIP-graph-captured) gradient buffers are zeroed in place HERE, on the
                # side stream behind the kernels that read them and before the bucket's event:
                # the next forward / graph replay waits for that event before it accumulates
                # into them again.  Zeroing them on the compute stream would race the step.
                if persistent:
                    torch._foreach_zero_(persistent)
                ov.bucket_done(key)
        for g in self.fp16_groups:  # the side stream still reads the gradients
            for p in g:
                if p.grad is not None:
                    p.grad.record_stream(ov.stream)
        self.zero_grad(skip_persistent=True)

    # ----------------------------------------------------------------- steps
    def zero_grad(self, set_to_none=True, skip_persistent=False):
        """skip_persistent: the persistent buffers were already zeroed on the overlapped step's
        side stream (_overlapped_fused_step); that holds until the next backward."""
        skip_persistent = skip_persistent or self._persistent_zeroed
        if skip_persistent:
            self._persistent_zeroed = True
        elif self._overlap is not None and self._overlap._done is not None:
            # an overlapped step may still read the persistent buffers on its side stream: order
            # the in-place zeroing after it (a stream wait, no host sync)
            torch.cuda.current_stream().wait_event(self._overlap._done)
        keep = []
        for group in self.fp16_groups:
            for p in group:
                if getattr(p, "_dsa_persistent_grad", False) and p.grad is not None:
                    if not skip_persistent:
                        keep.append(p.grad)  # a captured HIP graph accumulates into this buffer
                elif set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.detach_()
                    p.grad.zero_()
        if keep:
            from ...ops import wgrad_batch  # layer-stacked gradients: one fill per stack
            keep = wgrad_batch.zero_stacks(keep)
            if keep:
                torch._foreach_zero_(keep)

    def mark_new_gradients(self):
        """A backward that did not go through backward() (the pipeline engine's autograd calls)
        accumulated into the persistent buffers: the next zero_grad must zero them again."""
        self._persistent_zeroed = False

    def backward(self, loss, retain_graph=False):
        self.mark_new_gradients()
        (loss.float() * self.loss_scale).backward(retain_graph=retain_graph)

    def step(self, closure=None):
        params = [p for g in self.fp16_groups for p in g]
        if self._sync_free(params):
            coef_t = self._device_coef(params)
            if self._dev_skipped is None:
                self._dev_skipped = torch.zeros(1, dtype=torch.int32, device=coef_t.device)
            self._dev_skipped.add_(torch.isfinite(coef_t).logical_not())  # read lazily
            self.overflow = False
            if self._overlap is not None:
                self._overlapped_fused_step(coef_t)
                return self.overflow
            grads, outs = [], []
            for lp_group in self.fp16_groups:
                grads.append([p.grad for p in lp_group])
                outs.append([p.data for p in lp_group])
            self.optimizer.step(grads=grads, output_params=outs, scale=1.0, scale_tensor=coef_t)
            self.zero_grad()
            return self.overflow
        # one multi-tensor reduction gives both the global norm and the overflow flag (the sum
        # of squares is inf/nan iff some gradient entry is): no per-tensor isinf/isnan passes
        sq = grad_norm_sq_tensor(params, mpu=self.mpu).item()
        self.overflow = not math.isfinite(sq)
        prev = self.loss_scale
        if self.dynamic_loss_scale or self.overflow:
            self.loss_scaler.update_scale(self.overflow)
        if self.overflow:
            logger.info(f"[deepspeed] fp16 dynamic loss scale overflow! Skipping step. Attempted loss scale: "
                        f"{prev}, reducing to {self.loss_scale}")
            self.zero_grad()
            return self.overflow
        norm = math.sqrt(sq) / prev
        self._global_grad_norm = norm
        coef = 1.0 / prev
        if self.clip_grad > 0 and norm > self.clip_grad:
            coef *= self.clip_grad / (norm + 1e-6)
        if self._overlap is not None:
            self._overlapped_fused_step(torch.full((1,), coef, dtype=torch.float32, device=params[0].device))
            return self.overflow
        if getattr(self.optimizer, "supports_fused_lp_step", False):
            # fused LAMB: low-precision grads read with the unscale/clip factor folded in, the
            # updated master written back to the low-precision params by the same kernel
            grads, outs = [], []
            for lp_group, fp_group in zip(self.fp16_groups, self.fp32_groups):
                grads.append([p.grad for p in lp_group])
                outs.append([p.data for p in lp_group])
            self.optimizer.step(grads=grads, output_params=outs, scale=1.0 / coef)
            self.zero_grad()
            return self.overflow
        for lp_group, fp_group in zip(self.fp16_groups, self.fp32_groups):
            for p, m in zip(lp_group, fp_group):
                if p.grad is None:
                    m.grad = None
                    continue
                m.grad = p.grad.detach().float().mul_(coef)
        self.optimizer.step()
        for lp_group, fp_group in zip(self.fp16_groups, self.fp32_groups):
            for p, m in zip(lp_group, fp_group):
                m.grad = None
                p.data.copy_(m.data)
        self.zero_grad()
        return self.overflow

    # ----------------------------------------------------------------- checkpoints
    def state_dict(self):
        self.synchronize_step()
        return {"dynamic_loss_scale": self.dynamic_loss_scale, "cur_scale": self.loss_scale,
                "loss_scaler": self.loss_scaler.state_dict(), "overflow": self.overflow,
                "optimizer_state_dict": self.optimizer.state_dict(),
                "fp32_groups": [[m.detach().cpu() for m in g] for g in self.fp32_groups]}

    def load_state_dict(self, sd, load_optimizer_states=True):
        self.synchronize_step()
        self.dynamic_loss_scale = sd.get("dynamic_loss_scale", self.dynamic_loss_scale)
        if "loss_scaler" in sd:
            self.loss_scaler.load_state_dict(sd["loss_scaler"])
        self.overflow = sd.get("overflow", False)
        if load_optimizer_states:
            self.optimizer.load_state_dict(sd["optimizer_state_dict"])
        for cur, saved in zip(self.fp32_groups, sd["fp32_groups"]):
            for m, s in zip(cur, saved):
                m.data.copy_(s.to(m.device))
        for lp_group, fp_group in zip(self.fp16_groups, self.fp32_groups):
            for p, m in zip(lp_group, fp_group):
                p.data.copy_(m.data)

    def refresh_fp32_params(self):
        self.synchronize_step()
        for lp_group, fp_group in zip(self.fp16_groups, self.fp32_groups):
            for p, m in zip(lp_group, fp_group):
                m.data.copy_(p.data.float())
