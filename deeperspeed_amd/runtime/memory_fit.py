"""Measured HBM fitting for ZeRO-3 trainers (used by bench.py; usable by any training loop).

The static planner (bench.plan_memory) decides what must be true for a step to fit at all
(offload mode, activation recompute, micro-batch x grad-accum).  The two ZeRO-3 knobs that only
buy speed -- gathered-parameter retention (`stage3_max_live_parameters`, 2 B per retained bf16
element) and resident unit gradients (`resident_grads`, one bf16 copy of the model's gradients)
-- are NOT taken from a formula: the first step runs lean (no retention, no resident grads), the
headroom it leaves below the HBM limit is granted to retention first (it saves 2*GA-1 of the
2*GA per-step all-gathers), then to resident gradients (GA-1 of GA reduce-scatters).  Every later
warmup step is checked against the limit, and an overshoot is given back in the reverse order of
value: retention, then resident gradients, then the micro-batch is halved (GA doubled, same
tokens per step).  The policy is pure arithmetic over `FitState`; `apply()` maps its actions onto
a DeepSpeedEngine."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple


@dataclass
class FitState:
    params: int                  # model parameters (elements)
    world: int                   # data-parallel ranks
    micro_batch: int
    grad_accum: int
    live: int = 0                # stage3_max_live_parameters (elements)
    resident: bool = False
    auto_live: bool = True       # False: the user fixed it, never touched
    auto_resident: bool = True
    shard_grad_bytes_fp32: int = 4  # reduced-shard gradient bytes/param without resident grads (GA > 1)
    actions: List[Tuple[str, object]] = field(default_factory=list)

    # ------------------------------------------------------------------ costs (bytes)
    def resident_cost(self) -> int:
        """Extra HBM of resident gradients: full bf16 unit gradients for the whole model, minus
        the reduced shard shrinking from fp32 to bf16 (one reduction per step)."""
        saved = (self.shard_grad_bytes_fp32 - 2) * self.params // self.world if self.grad_accum > 1 else 0
        return 2 * self.params - saved

    def resident_useful(self) -> bool:
        return self.world > 1 and self.grad_accum > 1


# Allocator slack charged on every grant: the retained units and resident gradient buffers are
# many differently sized blocks allocated between the step's activations, and the caching
# allocator's reserved bytes grow past the allocated ones.  Measured on the full-depth emulated
# N=8 rank of GPT-NeoX-20B (profiles/r6a_emulated_world_notes.md): 71.1 GiB more allocated, 85.6 GiB
# more reserved (+20 %); charging the allocated cost alone let the N=4 plan grant 67 GiB into 74.8
# GiB of headroom and run out of memory in the next forward.
GRANT_SLACK = 0.25


def grow(st: FitState, headroom: float, slack: float = GRANT_SLACK) -> List[Tuple[str, object]]:
    """Grant measured headroom (bytes) to retention, then resident gradients, each at its
    allocated cost times (1 + slack)."""
    acts = []
    head = float(headroom)
    f = 1.0 + float(slack)
    if st.auto_live and head > 0:
        live = int(min(head / (2 * f), st.params))
        if live > st.live:
            head -= 2 * f * (live - st.live)
            st.live = live
            acts.append(("live", live))
    if st.auto_resident and not st.resident and st.resident_useful() and head >= f * st.resident_cost():
        st.resident = True
        acts.append(("resident", True))
    st.actions += acts
    return acts


def shrink(st: FitState, over: float, min_micro_batch: int = 1) -> List[Tuple[str, object]]:
    """Give back `over` bytes: retention first, then resident gradients, then halve the
    micro-batch (activations ~ micro-batch).  Returns the actions taken (may not cover `over`
    when nothing is left to give)."""
    acts = []
    need = float(over)
    if need <= 0:
        return acts
    if st.live > 0 and st.auto_live:
        give = int(min(st.live, -(-need // 2)))
        st.live -= give
        need -= 2 * give
        acts.append(("live", st.live))
    if need > 0 and st.resident and st.auto_resident:
        st.resident = False
        need -= st.resident_cost()
        acts.append(("resident", False))
    if need > 0 and st.micro_batch % 2 == 0 and st.micro_batch // 2 >= min_micro_batch:
        st.micro_batch //= 2
        st.grad_accum *= 2
        acts.append(("batch", (st.micro_batch, st.grad_accum)))
    st.actions += acts
    return acts


def apply(engine, acts) -> bool:
    """Apply fit actions to a DeepSpeedEngine with a ZeRO-3 optimizer (at a step boundary).
    Returns True when the batch shape changed (the caller must rebuild its micro-batches)."""
    opt = engine.optimizer
    reshaped = False
    for kind, val in acts:
        if kind == "live":
            opt.set_max_live_parameters(val)
            opt.release_retained()
        elif kind == "resident":
            opt.set_resident_grads(val)
        elif kind == "batch":
            engine.set_batch_shape(*val)
            reshaped = True
    return reshaped


class TierShortfall(RuntimeError):
    """The three moment tiers together cannot hold the model's Adam moments."""


def split_moment_tiers(blocks, budgets, bytes_per_param: int = 8):
    """Peak-parameter placement of Adam moments (offload_optimizer states='moments'): consecutive
    blocks of parameters (embedding, each layer, head) go to the first tier of ("gpu", "cpu",
    "nvme") -- HBM, pinned host memory, an aio-swapped file -- that still has room, so the
    fastest tiers fill first and a model whose moments exceed any one tier still trains.

    blocks: list of parameter lists; budgets: bytes per tier.  Returns (param groups with
    "moments_device", record); raises TierShortfall naming the shortfall when nothing fits."""
    order = ("gpu", "cpu", "nvme")
    left = {t: float(budgets.get(t, 0.0)) for t in order}
    groups = {t: [] for t in order}
    total = sum(p.numel() for ps in blocks for p in ps) * bytes_per_param
    for ps in blocks:
        need = float(bytes_per_param * sum(p.numel() for p in ps))
        tier = next((t for t in order if left[t] >= need), None)
        if tier is None:
            raise TierShortfall(
                f"moments do not fit: HBM {budgets.get('gpu', 0) / 2**30:.1f} + host {budgets.get('cpu', 0) / 2**30:.1f}"
                f" + disk {budgets.get('nvme', 0) / 2**30:.1f} GiB for {total / 2**30:.1f} GiB of moments; the next "
                f"block needs {need / 2**30:.2f} GiB, {(need - max(left.values())) / 2**30:.2f} GiB more than any "
                f"tier has left")
        left[tier] -= need
        groups[tier] += list(ps)
    rec = {t: {"params": sum(p.numel() for p in groups[t]),
               "gib": round(bytes_per_param * sum(p.numel() for p in groups[t]) / 2**30, 1)} for t in order}
    rec["budget_gib"] = {k: round(float(budgets.get(t, 0)) / 2**30, 1)
                         for k, t in (("hbm", "gpu"), ("host", "cpu"), ("disk", "nvme"))}
    return [{"params": groups[t], "moments_device": t} for t in order if groups[t]], rec
