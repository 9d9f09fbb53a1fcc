#!/usr/bin/env python
"""Consolidate ZeRO (stage 1/2/3) optimizer shards into one fp32 state dict, offline.

Reference parity: deepspeed/utils/zero_to_fp32.py (copied into every ZeRO checkpoint tag
directory; `python zero_to_fp32.py <checkpoint_dir> <output_file>`).  This version reads the
flat-arena layout signature stored in each `*_optim_states.pt` (bucket offsets, per-rank
chunking, parameter order) together with `param_shapes`, so it works for every stage and any
data-parallel world size.  Standalone on purpose: needs only torch.
"""

import argparse
import glob
import os
import re
from collections import OrderedDict

import torch


def get_optim_files(checkpoint_dir):
    files = glob.glob(os.path.join(checkpoint_dir, "*_optim_states.pt"))
    if not files:
        raise FileNotFoundError(f"can't find '*_optim_states.pt' files in directory '{checkpoint_dir}'")

    def rank_of(f):
        m = re.search(r"zero_pp_rank_(\d+)_", os.path.basename(f))
        return int(m.group(1)) if m else 0

    return sorted(files, key=rank_of)


REFERENCE_KEYS = {1: "local_sub_partitions_of_fp32_groups", 2: "single_partition_of_fp32_groups",
                  3: "fp32_flat_groups"}


class _PickledScaler:
    """Stand-in for the loss-scaler object reference checkpoints pickle (attributes only)."""


_SAFE = [(_PickledScaler, "deepspeed.runtime.fp16.loss_scaler.DynamicLossScaler"),
         (_PickledScaler, "deepspeed.runtime.fp16.loss_scaler.LossScaler")]


def _load(f):
    with torch.serialization.safe_globals(_SAFE):
        return torch.load(f, map_location="cpu", weights_only=True)


def parse_optim_states(files):
    sds = [_load(f) for f in files]
    osds = [sd["optimizer_state_dict"] for sd in sds]
    if "layout" not in osds[0]:
        return _parse_reference(sds, osds)
    key = osds[0]["fp32_groups_key"]
    zero_stage = osds[0].get("zero_stage", 0)
    world = osds[0].get("partition_count", len(osds))
    if world != len(osds):
        raise ValueError(f"Expected {world} optimizer shards, found {len(osds)}")
    shards = [o[key] for o in osds]
    return zero_stage, world, shards, osds[0]["layout"], sds[0]["param_shapes"]


def _parse_reference(sds, osds):
    """Reference-layout (DeepSpeed 0.3.15) checkpoint -- written by the reference or by this
    framework with checkpoint.zero_format = "reference".  Returns per-group lists of full fp32
    parameters in optimizer-group order, and the names to give them.

    The reference script (zero_to_fp32.py:70-151) reads only param group 0 and assumes it holds
    every module parameter in module order.  Here every group is read; with several groups the
    file must record which parameter is where (`dsa_group_param_names`), otherwise the groups
    cannot be mapped onto `param_shapes` (module order) and this raises instead of guessing."""
    stage = osds[0].get("zero_stage", 0)
    if stage not in REFERENCE_KEYS:
        raise ValueError(f"reference checkpoint of zero stage {stage} cannot be consolidated")
    world = osds[0].get("partition_count", len(osds))
    if world != len(osds):
        raise ValueError(f"Expected {world} optimizer shards, found {len(osds)}")
    shapes = sds[0]["param_shapes"]
    shapes = shapes[0] if isinstance(shapes, list) else shapes
    group_names = sds[0].get("dsa_group_param_names")
    key = REFERENCE_KEYS[stage]
    if stage == 3:
        pgs = osds[0].get("optimizer_state_dict", {}).get("param_groups")
        nflat = len(osds[0][key])
        subs = [list(pg["params"]) for pg in pgs] if pgs and all("params" in pg for pg in pgs) else [list(range(nflat))]
    else:
        subs = [[g] for g in range(len(osds[0][key]))]
    if group_names is None:
        if len(subs) > 1:
            raise ValueError(f"checkpoint has {len(subs)} optimizer param groups but does not record which "
                             f"parameters each holds; param_shapes is in module order, so the groups cannot "
                             f"be mapped back (save with checkpoint.zero_format=reference from this framework)")
        group_names = [list(shapes.keys())]
    out_groups = []
    for G, names in enumerate(group_names):
        numels = [_numel(shapes[n]) for n in names]
        if stage == 2:
            flat = torch.cat([o[key][G].reshape(-1).float() for o in osds])
        elif stage == 1:
            intervals = len(osds[0][key][G])
            flat = torch.cat([osds[r][key][G][c].reshape(-1).float() for c in range(intervals) for r in range(world)])
        if stage in (1, 2):
            params, off = [], 0
            for n in numels:
                params.append(flat[off: off + n])
                off += n
            if off > flat.numel():
                raise ValueError(f"group {G}: shards hold {flat.numel()} elements, its parameters need {off}")
        else:
            per_rank = [torch.cat([o[key][k].reshape(-1).float() for k in subs[G]]) for o in osds]
            params, off = [], 0
            for n in numels:
                part, _ = zero3_partitioned_param_info(n, world)
                params.append(torch.cat([t[off: off + part] for t in per_rank])[:n])
                off += part
        out_groups.append(list(zip(names, params)))
    return stage, world, out_groups, None, shapes


def _numel(shape):
    n = 1
    for d in shape:
        n *= int(d)
    return n


def _reference_state_dict(groups, shapes):
    found = {name: t for grp in groups for name, t in grp}
    out = OrderedDict()
    for name, shape in shapes.items():  # module order, like the reference's output
        if name not in found:
            raise ValueError(f"parameter {name} is in param_shapes but in no optimizer group")
        out[name] = found[name].view(*shape).clone()
    return out


def _group_params(shards_of_group, sig):
    out = {}
    for b in sig["buckets"]:
        full = torch.cat([s[b["shard_offset"]: b["shard_offset"] + b["chunk"]] for s in shards_of_group])
        for pi, off, n in zip(b["pidx"], b["offsets"], b["numels"]):
            out[pi] = full[off: off + n]
    return out


def convert_zero_chkpt_to_fp32_consolid_state_dict(checkpoint_dir, output_file):
    print(f"Processing zero checkpoint '{checkpoint_dir}'")
    stage, world, shards, layout, param_shapes = parse_optim_states(get_optim_files(checkpoint_dir))
    print(f"Detected checkpoint of type zero stage {stage}, world_size: {world}")
    if layout is None:
        state_dict = _reference_state_dict(shards, param_shapes)
        print(f"Saving fp32 state dict to {output_file} ({len(state_dict)} tensors, reference layout)")
        torch.save(state_dict, output_file)
        return state_dict
    state_dict = OrderedDict()
    for gi, sig in enumerate(layout):
        flat = _group_params([s[gi] for s in shards], sig)
        names = list(param_shapes[gi].keys())
        for pi, name in enumerate(names):
            shape = param_shapes[gi][name]
            n = 1
            for d in shape:
                n *= d
            t = flat[pi]
            assert t.numel() == n, f"{name}: {t.numel()} != {n}"
            state_dict[name] = t.view(*shape).clone()
    print(f"Saving fp32 state dict to {output_file} ({len(state_dict)} tensors)")
    torch.save(state_dict, output_file)
    return state_dict


def zero3_partitioned_param_info(unpartitioned_numel, world_size):
    """(per-rank partition, padding) of one ZeRO-3 parameter.  The reference's version floors
    the partition (zero_to_fp32.py:63-67) and mis-reads any parameter whose size is not a
    multiple of the world size; the partition is ceil(numel / world) (partition_parameters.py)."""
    remainder = unpartitioned_numel % world_size
    padding_numel = (world_size - remainder) if remainder else 0
    partitioned_numel = (unpartitioned_numel + padding_numel) // world_size
    return partitioned_numel, padding_numel


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("checkpoint_dir", type=str,
                        help="path to the deepspeed checkpoint folder, e.g., path/checkpoint-1/global_step1")
    parser.add_argument("output_file", type=str,
                        help="path to the pytorch fp32 state_dict output file (e.g. path/pytorch_model.bin)")
    args = parser.parse_args()
    convert_zero_chkpt_to_fp32_consolid_state_dict(args.checkpoint_dir, args.output_file)
