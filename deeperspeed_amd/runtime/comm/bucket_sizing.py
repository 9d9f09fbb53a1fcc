"""Collective bucket sizes for RCCL over xGMI ("auto" values of the ZeRO bucket keys).

The reference picks fixed element counts (`reduce_bucket_size` / `allgather_bucket_size` 5e8,
`stage3_prefetch_bucket_size` 5e7, deepspeed/runtime/zero/constants.py) tuned for NVLink /
NVSwitch.  On an MI355X node every GPU reaches the other seven over point-to-point xGMI links and
RCCL runs its rings over them, so a ring collective over N ranks of B bytes costs about

    t(B) = 2 (N - 1) * alpha  +  (N - 1) / N * B / beta

with alpha the per-step latency (launch + flag handshake, a few microseconds) and beta the
per-rank ring bandwidth (bounded by the links one rank drives).  The smallest bucket whose
latency term stays within `overhead` of the bandwidth term is

    B >= 2 N alpha beta / overhead,

and anything larger only adds memory (every in-flight bucket is a full-size buffer) and delays
the first overlap with compute.  The defaults below (alpha 10 us, beta 300 GB/s, overhead 10 %)
give 48 MB at N = 2 and 192 MB at N = 8 -- 96M bf16 elements at 8 ranks, a fifth of the
reference's 5e8 default -- and the sizes are clamped to [4M, 5e8] elements.  At N = 1 (no
collective) the reference default is kept.
"""

from __future__ import annotations

import os

DEFAULT_ALPHA_S = 10e-6
DEFAULT_BETA_BPS = 300e9
DEFAULT_OVERHEAD = 0.10
MIN_ELEMS = 1 << 22
MAX_ELEMS = int(5e8)


def ring_time_s(nbytes: float, world: int, alpha: float = DEFAULT_ALPHA_S, beta: float = DEFAULT_BETA_BPS) -> float:
    """Modelled time of one ring reduce-scatter (or all-gather) of `nbytes` over `world` ranks."""
    if world <= 1:
        return 0.0
    return 2 * (world - 1) * alpha + (world - 1) / world * nbytes / beta


def auto_bucket_elems(world: int, elem_size: int = 2, alpha: float = None, beta: float = None,
                      overhead: float = DEFAULT_OVERHEAD) -> int:
    """Bucket size in elements for `world` ranks (env DSA_XGMI_ALPHA_US / DSA_XGMI_GBPS override the
    link model)."""
    if world <= 1:
        return MAX_ELEMS
    alpha = alpha if alpha is not None else float(os.environ.get("DSA_XGMI_ALPHA_US", DEFAULT_ALPHA_S * 1e6)) * 1e-6
    beta = beta if beta is not None else float(os.environ.get("DSA_XGMI_GBPS", DEFAULT_BETA_BPS / 1e9)) * 1e9
    nbytes = 2.0 * world * alpha * beta / overhead
    return int(min(MAX_ELEMS, max(MIN_ELEMS, nbytes // elem_size)))


def resolve(value, world: int, elem_size: int = 2, scale: float = 1.0) -> int:
    """An int bucket size as configured, or the modelled size for the string "auto"
    (`scale` < 1 for the prefetch window, which the reference keeps 10x smaller)."""
    if isinstance(value, str):
        if value.strip().lower() != "auto":
            return int(float(value))
        return max(MIN_ELEMS, int(auto_bucket_elems(world, elem_size) * scale))
    return int(value)
