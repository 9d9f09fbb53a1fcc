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


REFERENCE_KEYS = {2: "single_partition_of_fp32_groups", 3: "fp32_flat_groups"}


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
    """Reference (DeepSpeed 0.3.15) checkpoint: contiguous per-group partitions, `param_shapes`
    = every module parameter in order (reference zero_to_fp32.py:70-151; that script reads
    only the first group / sub-group, this one all of them)."""
    stage = osds[0].get("zero_stage", 0)
    if stage not in REFERENCE_KEYS:
        raise ValueError(f"reference checkpoint of zero stage {stage}: only stage 2 and 3 can be consolidated")
    world = osds[0].get("partition_count", len(osds))
    if world != len(osds):
        raise ValueError(f"Expected {world} optimizer shards, found {len(osds)}")
    # every param group (stage 2) / sub-group (stage 3) of a rank, in order: consecutive
    # parameters, so their concatenation is the rank's range of every parameter in turn
    shards = [torch.cat([t.reshape(-1).float() for t in o[REFERENCE_KEYS[stage]]]) for o in osds]
    shapes = sds[0]["param_shapes"]
    shapes = shapes[0] if isinstance(shapes, list) else shapes
    return stage, world, shards, None, shapes


def _reference_state_dict(stage, world, shards, shapes):
    out = OrderedDict()
    flat = torch.cat(shards) if stage == 2 else None
    off = 0
    for name, shape in shapes.items():
        n = 1
        for d in shape:
            n *= d
        if stage == 2:
            out[name] = flat[off: off + n].view(*shape).clone()
            off += n
        else:
            part, _ = zero3_partitioned_param_info(n, world)
            out[name] = torch.cat([s[off: off + part] for s in shards])[:n].view(*shape).clone()
            off += part
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
        state_dict = _reference_state_dict(stage, world, shards, param_shapes)
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
