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


# ---------------------------------------------------------------------------- export
def _ceil_div(a, b):
    return -(-a // b)


def _stage1_geometry(total: int, world: int, max_elems_per_comm: int):
    """(sub_partition_size, num_comm_intervals) exactly as the reference computes them
    (stage1.py:314-343 best_max_elems_per_comm, :580-610 sub-partition alignment)."""
    mepc = int(max_elems_per_comm)
    max_iv = _ceil_div(total, mepc)
    pad_max = mepc * max_iv - total
    min_iv = total // mepc
    if min_iv > 0:
        pad_min = _ceil_div(total, world * min_iv)
        if pad_max > pad_min:
            mepc = pad_min + mepc
    part = _ceil_div(total, world)
    comm_part = int(mepc // world)
    if part <= comm_part:
        return part, 1
    return comm_part, _ceil_div(part, comm_part)


def _reference_ranges(stage: int, numels: Sequence[int], world: int, rank: int, max_elems_per_comm: int,
                      sub_group_size: int):
    """Where this rank's reference-layout pieces come from.  Returns a list of flat tensors
    (stage 1: one per comm interval; stage 2: one; stage 3: one per sub-group), each a list of
    (param j, start in param, length) runs -- plus, for stage 3, zero-padding lengths (None j)."""
    offs, acc = [], 0
    for n in numels:
        offs.append(acc)
        acc += n
    total = acc

    def runs(lo, hi):
        out = []
        for j, (o, n) in enumerate(zip(offs, numels)):
            a, b = max(lo, o), min(hi, o + n)
            if a < b:
                out.append((j, a - o, b - a))
        return out

    if stage == 2:
        part = _ceil_div(total, world)
        return [runs(rank * part, min((rank + 1) * part, total))]
    if stage == 1:
        sps, intervals = _stage1_geometry(total, world, max_elems_per_comm)
        return [runs((c * world + rank) * sps, min((c * world + rank + 1) * sps, total)) for c in range(intervals)]
    # stage 3: per-parameter ceil(n / world) ranges, padded, grouped into sub-groups
    subs, cur, cur_n = [], [], 0
    for j, n in enumerate(numels):
        ps = _ceil_div(n, world)
        lo = min(rank * ps, n)
        hi = min((rank + 1) * ps, n)
        if hi > lo:
            cur.append((j, lo, hi - lo))
        if ps - (hi - lo) > 0:
            cur.append((None, 0, ps - (hi - lo)))
        cur_n += ps
        if (sub_group_size is not None and cur_n >= sub_group_size) or j == len(numels) - 1:
            subs.append(cur)
            cur, cur_n = [], 0
    if sum(_ceil_div(n, world) for n in numels) <= (sub_group_size or 0) or sub_group_size is None:
        # the reference keeps one sub-group when the whole group fits (stage3.py:1337-1338)
        subs = [[r for s in subs for r in s]]
    return subs


def _assemble(runs, full: Dict[int, torch.Tensor]) -> torch.Tensor:
    parts = [torch.zeros(ln) if j is None else full[j][st: st + ln] for j, st, ln in runs]
    return torch.cat(parts) if parts else torch.zeros(0)


def export_reference_state_dict(opt, max_elems_per_comm: int = int(5e8), sub_group_size: int = int(1e12),
                                comm_device=None) -> dict:
    """This rank's optimizer state in the reference (DeepSpeed 0.3.15) ZeRO-1/2/3 layout.

    Collective over the data-parallel group: every bucket's fp32 master and Adam moments are
    all-gathered one bucket at a time (the flat-arena shards interleave every bucket over the
    ranks, the reference gives each rank one contiguous range), and each rank keeps only the
    parameters its reference range touches.  Written keys mirror the reference exactly:
    `single_partition_of_fp32_groups` + lean `base_optimizer_state` (stage 2, stage2.py:
    1720-1751), `local_sub_partitions_of_fp32_groups` + per-interval lean states +
    `num_comm_intervals_per_group` (stage 1, stage1.py:924-943), `fp32_flat_groups` + a torch
    `optimizer_state_dict` over the sub-group flats (stage 3, stage3.py:3046-3059)."""
    import torch.distributed as dist
    stage = opt._zero_stage()
    if stage not in (1, 2, 3):
        raise ValueError(f"reference-layout export needs ZeRO stage 1-3 (got {stage})")
    world, rank = opt._layout_world_rank()
    group = opt.dp_group
    dev = comm_device
    if dev is None:
        dev = opt.device if (dist.is_initialized() and dist.get_backend(group) == "nccl") else torch.device("cpu")
    orig = opt._orig_group_params
    where = {}  # id(p) -> (group index, position j)
    for G, plist in enumerate(orig):
        for j, p in enumerate(plist):
            where[id(p)] = (G, j)
    numels = [[p.ds_numel if hasattr(p, "ds_numel") else p.numel() for p in plist] for plist in orig]
    plans = [_reference_ranges(stage, numels[G], world, rank, max_elems_per_comm, sub_group_size)
             for G in range(len(orig))]
    needed = [{j for flat in plans[G] for j, _, _ in flat if j is not None} for G in range(len(orig))]
    names = ("master", "exp_avg", "exp_avg_sq")
    full = {n: [dict() for _ in orig] for n in names}
    steps = [0] * len(orig)
    for gi, g in enumerate(opt.groups):
        shards = {"master": opt.master_fp32(g).float()}
        st = opt.optimizer.state.get(g.master, {}) if g.master is not None else {}
        for n in ("exp_avg", "exp_avg_sq"):
            t = opt._nvme_read_group(gi, n) if opt.nvme else st.get(n)
            shards[n] = t.detach().float().cpu() if torch.is_tensor(t) else torch.zeros(g.shard_numel)
        steps[g.group_index] = int(st.get("step", steps[g.group_index]) or 0) if st else steps[g.group_index]
        for b in g.buckets:
            keep = [i for i, p in enumerate(b.params) if where[id(p)][1] in needed[where[id(p)][0]]]
            for n in names:
                chunk = shards[n][b.shard_offset: b.shard_offset + b.chunk].to(dev)
                out = torch.empty(b.numel, dtype=torch.float32, device=dev)
                if world > 1:
                    dist.all_gather_into_tensor(out, chunk, group=group)
                else:
                    out.copy_(chunk)
                out = out.cpu()
                for i in keep:
                    G, j = where[id(b.params[i])]
                    full[n][G][j] = out[b.offsets[i]: b.offsets[i] + b.numels[i]].clone()
    sd = {"loss_scaler": opt.loss_scaler.state_dict(), "dynamic_loss_scale": opt.dynamic_loss_scale,
          "overflow": opt.overflow, "zero_stage": stage, "partition_count": world}
    hyper = [{k: v for k, v in pg.items() if k != "params"} for pg in opt.optimizer.param_groups]
    if stage == 2:
        sd["single_partition_of_fp32_groups"] = [_assemble(plans[G][0], full["master"][G]) for G in range(len(orig))]
        sd["base_optimizer_state"] = [{"step": steps[G],
                                       "exp_avg": _assemble(plans[G][0], full["exp_avg"][G]),
                                       "exp_avg_sq": _assemble(plans[G][0], full["exp_avg_sq"][G])}
                                      for G in range(len(orig))]
    elif stage == 1:
        sd["local_sub_partitions_of_fp32_groups"] = [[_assemble(r, full["master"][G]) for r in plans[G]]
                                                     for G in range(len(orig))]
        sd["base_optimizer_state"] = [[{"step": steps[G], "exp_avg": _assemble(r, full["exp_avg"][G]),
                                        "exp_avg_sq": _assemble(r, full["exp_avg_sq"][G])} for r in plans[G]]
                                      for G in range(len(orig))]
        sd["num_comm_intervals_per_group"] = [len(plans[G]) for G in range(len(orig))]
    else:
        flats, state, pgs, k = [], {}, [], 0
        for G in range(len(orig)):
            ids = []
            for r in plans[G]:
                flats.append(_assemble(r, full["master"][G]))
                state[k] = {"step": steps[G], "exp_avg": _assemble(r, full["exp_avg"][G]),
                            "exp_avg_sq": _assemble(r, full["exp_avg_sq"][G])}
                ids.append(k)
                k += 1
            pgs.append(dict(hyper[G] if G < len(hyper) else {}, params=ids))
        sd["fp32_flat_groups"] = flats
        sd["optimizer_state_dict"] = {"state": state, "param_groups": pgs}
    return sd


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
