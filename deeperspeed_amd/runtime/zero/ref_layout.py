"""Import of reference-layout (DeepSpeed 0.3.15 / DeeperSpeed) ZeRO optimizer checkpoints.

The reference shards every optimizer param group as ONE contiguous flat tensor of the
group's parameters in registration order, and saves per data-parallel rank:

* ZeRO-1 (stage1.py:356-401, 857-899, 924-943): the flat group padded to
  `num_comm_intervals * dp` sub-partitions; sub-partition `c * dp + r` belongs to rank r
  (comm interval c).  Saved: `local_sub_partitions_of_fp32_groups[g] = [sub-partition of
  interval c for c ...]` and `base_optimizer_state[g] = [lean state per sub-partition]`,
  padding removed.
* ZeRO-2 (stage2.py:200-250, 593-611, 1150-1168, 1687-1745): the flat group padded to a
  multiple of dp, split into dp equal ranges.  Saved: `single_partition_of_fp32_groups[g]`
  (rank's range, tail padding removed on the last rank) and `base_optimizer_state[g]`
  (lean {exp_avg, exp_avg_sq, step}).
* ZeRO-3 (stage3.py:1332-1356, 3046-3060; partition_parameters.py:547-553, 610-690): every
  parameter is padded to a multiple of dp and split into dp ranges of ceil(numel/dp); a
  rank's flat sub-group is the concatenation of its range of every parameter of the
  sub-group.  Saved: `fp32_flat_groups[k]` per sub-group (padding kept) and a torch
  `optimizer_state_dict` whose param k is sub-group k's flat tensor.

This framework's own shards are interleaved per bucket (layout.py) and carry a `layout`
signature plus `dsa_layout_version`; the fp32 shards are stored under a different key than
the reference's, so reference tools fail loudly on them instead of mis-reading them.
`merge_reference_shards` turns any of the three reference formats into full per-parameter
fp32 tensors (masters and Adam moments), which the optimizer then re-partitions into its
own layout for the current world size.
"""

from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch

REF_FP32_KEYS = {1: "local_sub_partitions_of_fp32_groups", 2: "single_partition_of_fp32_groups",
                 3: "fp32_flat_groups"}
LAYOUT_VERSION = 2  # 1: round-1 files (reference key names + layout signature); 2: own key


def is_reference_layout(sd: dict) -> bool:
    return "layout" not in sd and any(k in sd for k in REF_FP32_KEYS.values())


def _split(flat: torch.Tensor, numels: Sequence[int]) -> List[torch.Tensor]:
    out, off = [], 0
    for n in numels:
        out.append(flat[off: off + n])
        off += n
    if off > flat.numel():
        raise ValueError(f"reference shard holds {flat.numel()} elements, parameters need {off}")
    return out


def _cat_ranks(pieces: Sequence[torch.Tensor]) -> torch.Tensor:
    return torch.cat([p.reshape(-1).float() for p in pieces]) if pieces else torch.zeros(0)


def _merge_stage12(sds, stage, group_numels):
    key = REF_FP32_KEYS[stage]
    world = len(sds)
    masters, moments = [], []
    for g, numels in enumerate(group_numels):
        if stage == 2:
            flat = _cat_ranks([sd[key][g] for sd in sds])
            states = [sd["base_optimizer_state"][g] for sd in sds]
            mflat = {k: _cat_ranks([s[k] for s in states]) for k in ("exp_avg", "exp_avg_sq")
                     if all(torch.is_tensor(s.get(k)) for s in states)}
            step = states[0].get("step", 0)
        else:
            intervals = len(sds[0][key][g])
            order = [(c, r) for c in range(intervals) for r in range(world)]
            flat = _cat_ranks([sds[r][key][g][c] for c, r in order])
            states = [[sd["base_optimizer_state"][g][c] for c in range(intervals)] for sd in sds]
            mflat = {k: _cat_ranks([states[r][c][k] for c, r in order]) for k in ("exp_avg", "exp_avg_sq")
                     if all(torch.is_tensor(states[r][c].get(k)) for c, r in order)}
            step = states[0][0].get("step", 0) if intervals else 0
        masters.append(_split(flat, numels))
        moments.append({"step": step, **{k: _split(v, numels) for k, v in mflat.items()}})
    return masters, moments


def _merge_stage3(sds, group_numels):
    """Per-parameter reassembly of ZeRO-3 sub-groups; sub-group boundaries are recovered from
    the flat lengths (the reference does not store sub_group_size)."""
    world = len(sds)
    flats = [sd[REF_FP32_KEYS[3]] for sd in sds]
    opt_states = [sd.get("optimizer_state_dict", {}).get("state", {}) for sd in sds]
    part = [[-(-n // world) for n in numels] for numels in group_numels]
    masters = [[None] * len(n) for n in group_numels]
    moments = [{"step": 0} for _ in group_numels]
    g, j = 0, 0  # next (group, param) to assign
    for k in range(len(flats[0])):
        length = flats[0][k].numel()
        if g >= len(group_numels):
            raise ValueError("reference ZeRO-3 checkpoint has more sub-groups than the model has param groups")
        members, acc = [], 0
        while acc < length:
            if j >= len(part[g]):
                raise ValueError(f"reference sub-group {k} ({length} elements) does not align with param group {g}")
            members.append(j)
            acc += part[g][j]
            j += 1
        if acc != length:
            raise ValueError(f"reference sub-group {k}: {length} elements, parameters give {acc}")
        names = [("master", [f[k] for f in flats])]
        for mk in ("exp_avg", "exp_avg_sq"):
            if all(torch.is_tensor(st.get(k, {}).get(mk)) for st in opt_states):
                names.append((mk, [st[k][mk] for st in opt_states]))
        if opt_states[0].get(k, {}).get("step") is not None:
            moments[g]["step"] = opt_states[0][k]["step"]
        for name, per_rank in names:
            off = 0  # offset of the parameter's range inside every rank's flat sub-group
            for jj in members:
                ps, n = part[g][jj], group_numels[g][jj]
                full = _cat_ranks([t.reshape(-1)[off: off + ps] for t in per_rank])[:n]
                if name == "master":
                    masters[g][jj] = full
                else:
                    moments[g].setdefault(name, [None] * len(group_numels[g]))[jj] = full
                off += ps
        if j == len(part[g]):
            g, j = g + 1, 0
    for g, ms in enumerate(masters):
        if any(m is None for m in ms):
            raise ValueError(f"reference ZeRO-3 checkpoint does not cover every parameter of group {g}")
    return masters, moments


def merge_reference_shards(sds: Sequence[dict], group_numels: Sequence[Sequence[int]]
                           ) -> Tuple[List[List[torch.Tensor]], List[Dict]]:
    """Full per-parameter fp32 tensors from the saved optimizer states of every reference rank.

    `group_numels[g]` lists the element count of every parameter of optimizer param group g
    in registration order.  Returns (masters[g][j], moments[g] = {"step", "exp_avg": [...],
    "exp_avg_sq": [...]})."""
    stage = int(sds[0].get("zero_stage", 0))
    if stage not in REF_FP32_KEYS or REF_FP32_KEYS[stage] not in sds[0]:
        raise ValueError(f"not a reference ZeRO checkpoint (zero_stage={stage})")
    if int(sds[0].get("partition_count", len(sds))) != len(sds):
        raise ValueError(f"reference checkpoint was saved by {sds[0].get('partition_count')} ranks, "
                         f"{len(sds)} optimizer files given")
    if stage == 3:
        return _merge_stage3(sds, group_numels)
    return _merge_stage12(sds, stage, group_numels)
