"""Flat-arena parameter layout shared by every ZeRO stage.

This is the MI355X-first replacement for the reference's per-stage flattening logic
(stage1.py:203-287 sub-partitions, stage2.py:388-489 flat groups, stage3.py:1621-1690
sub-groups).  One layout object serves all stages:

* A *group* is one optimizer param group restricted to one (dtype, model-parallel) class.
* A group's parameters are packed into *buckets*; every bucket is a contiguous range of
  elements whose length is padded to a multiple of ``world * ALIGN``.  Each parameter
  starts on an ``ALIGN``-element (128-byte for bf16) boundary so every per-parameter
  view is vector-aligned for the HIP kernels and hipBLASLt.
* Sharding is *interleaved per bucket*: rank ``r`` owns chunk ``r`` (of ``numel/world``
  elements) of every bucket.  A rank's shard of the group is the concatenation of its
  chunks, so optimizer state (fp32 master, Adam moments, reduced gradients) is one
  contiguous tensor per group, while every collective is a single tensor-native RCCL call
  per bucket: ``reduce_scatter_tensor(shard_chunk, bucket)`` in backward and
  ``all_gather_into_tensor(bucket, shard_chunk)`` after the step / before use (ZeRO-3).
* Stages 1/2 build buckets by size (``reduce_bucket_size``) in reverse registration order
  so they fill in backward order; ZeRO-3 builds one bucket per (module unit, group).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

ALIGN = 64  # elements; 128 B for bf16, 256 B for fp32


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class Bucket:
    index: int  # position within the group
    params: List[torch.nn.Parameter]
    offsets: List[int]  # element offset of each param inside the bucket
    numels: List[int]
    numel: int  # padded bucket length (multiple of world*ALIGN)
    chunk: int  # numel // world
    arena_offset: int  # start inside the group arena (stages 0-2); -1 when not arena-backed
    shard_offset: int  # start of this rank's chunk inside the group shard tensors
    unit: Optional[object] = None  # ZeRO-3 unit owning this bucket

    def param_slice(self, i: int) -> Tuple[int, int]:
        return self.offsets[i], self.offsets[i] + self.numels[i]

    def chunk_overlap(self, rank: int, i: int) -> Optional[Tuple[int, int, int]]:
        """Intersection of param i with rank's chunk: (param_start, chunk_start, length) or None."""
        c0, c1 = rank * self.chunk, (rank + 1) * self.chunk
        p0, p1 = self.param_slice(i)
        lo, hi = max(c0, p0), min(c1, p1)
        if lo >= hi:
            return None
        return lo - p0, lo - c0, hi - lo


@dataclass
class FlatGroup:
    group_index: int  # index of the optimizer param group
    sub_index: int
    dtype: torch.dtype
    model_parallel: bool
    params: List[torch.nn.Parameter]
    buckets: List[Bucket] = field(default_factory=list)
    arena_numel: int = 0
    shard_numel: int = 0
    hyper: Dict = field(default_factory=dict)
    # runtime tensors attached by the optimizer
    arena: Optional[torch.Tensor] = None
    grad_arena: Optional[torch.Tensor] = None
    shard_param: Optional[torch.Tensor] = None
    shard_grad: Optional[torch.Tensor] = None
    master: Optional[torch.Tensor] = None

    def param_index(self):
        """map param -> (bucket, position)"""
        out = {}
        for b in self.buckets:
            for i, p in enumerate(b.params):
                out[p] = (b, i)
        return out


def _make_bucket(index, params, world, arena_offset, shard_offset, unit=None) -> Bucket:
    offs, nums, cur = [], [], 0
    for p in params:
        n = p.ds_numel if hasattr(p, "ds_numel") else p.numel()
        offs.append(cur)
        nums.append(n)
        cur = _round_up(cur + n, ALIGN)
    total = _round_up(max(cur, 1), world * ALIGN)
    return Bucket(index=index, params=list(params), offsets=offs, numels=nums, numel=total, chunk=total // world,
                  arena_offset=arena_offset, shard_offset=shard_offset, unit=unit)


def split_param_group(params: Sequence[torch.nn.Parameter], is_mp_fn) -> List[Tuple[torch.dtype, bool, list]]:
    """Split a param group by (dtype, model_parallel) keeping registration order."""
    keys: List[Tuple[torch.dtype, bool]] = []
    by_key: Dict[Tuple[torch.dtype, bool], list] = {}
    for p in params:
        if not p.requires_grad:
            continue
        k = (p.dtype, bool(is_mp_fn(p)))
        if k not in by_key:
            by_key[k] = []
            keys.append(k)
        by_key[k].append(p)
    return [(k[0], k[1], by_key[k]) for k in keys]


def build_size_buckets(group: FlatGroup, world: int, bucket_size: int) -> FlatGroup:
    """Stages 0-2: pack params (reverse order, i.e. backward order) into ~bucket_size buckets."""
    order = list(reversed(group.params))
    cur: List = []
    cur_n = 0
    arena_off = shard_off = 0
    blists = []
    for p in order:
        n = _round_up(p.ds_numel if hasattr(p, "ds_numel") else p.numel(), ALIGN)
        if cur and cur_n + n > bucket_size:
            blists.append(cur)
            cur, cur_n = [], 0
        cur.append(p)
        cur_n += n
    if cur:
        blists.append(cur)
    for i, plist in enumerate(blists):
        b = _make_bucket(i, plist, world, arena_off, shard_off)
        group.buckets.append(b)
        arena_off += b.numel
        shard_off += b.chunk
    group.arena_numel = arena_off
    group.shard_numel = shard_off
    return group


def build_unit_buckets(group: FlatGroup, world: int, unit_of_param) -> FlatGroup:
    """ZeRO-3: one bucket per (unit, group); units ordered by first appearance."""
    units: List = []
    by_unit: Dict[int, list] = {}
    for p in group.params:
        u = unit_of_param(p)
        if id(u) not in by_unit:
            by_unit[id(u)] = []
            units.append(u)
        by_unit[id(u)].append(p)
    shard_off = 0
    for i, u in enumerate(units):
        b = _make_bucket(i, by_unit[id(u)], world, -1, shard_off, unit=u)
        group.buckets.append(b)
        shard_off += b.chunk
    group.shard_numel = shard_off
    group.arena_numel = 0
    return group


def layout_signature(groups: Sequence[FlatGroup]) -> List[Dict]:
    """Serializable description of the layout (stored in ZeRO checkpoints so an elastic
    restore can rebuild full per-parameter tensors from any world size)."""
    out = []
    for g in groups:
        pos = {id(p): i for i, p in enumerate(g.params)}
        out.append({
            "group_index": g.group_index,
            "sub_index": g.sub_index,
            "buckets": [{"offsets": b.offsets, "numels": b.numels, "numel": b.numel, "chunk": b.chunk,
                         "shard_offset": b.shard_offset, "pidx": [pos[id(p)] for p in b.params]}
                        for b in g.buckets],
            "shard_numel": g.shard_numel,
        })
    return out


def shards_to_params(shards: Sequence[torch.Tensor], sig: Dict) -> Dict[int, torch.Tensor]:
    """Rebuild the flat (unpadded) contents of every parameter of one group from the
    shards of all ranks (list index = rank) using the saved layout signature.
    Returns {param position in group: flat tensor}."""
    out = {}
    for b in sig["buckets"]:
        full = torch.cat([s[b["shard_offset"]: b["shard_offset"] + b["chunk"]] for s in shards])
        for pi, off, n in zip(b["pidx"], b["offsets"], b["numels"]):
            out[pi] = full[off: off + n]
    return out


def params_to_shard(flat_params: Dict[int, torch.Tensor], group: FlatGroup, rank: int, dtype) -> torch.Tensor:
    """Inverse of shards_to_params for this rank under the *current* layout."""
    shard = torch.zeros(group.shard_numel, dtype=dtype)
    pos = {id(p): i for i, p in enumerate(group.params)}
    for b in group.buckets:
        for i, p in enumerate(b.params):
            ov = b.chunk_overlap(rank, i)
            src = flat_params[pos[id(p)]]
            if ov is None:
                continue
            p0, c0, ln = ov
            shard[b.shard_offset + c0: b.shard_offset + c0 + ln].copy_(src[p0: p0 + ln])
    return shard
