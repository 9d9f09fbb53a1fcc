"""Writing ZeRO checkpoints in the REFERENCE layout (`checkpoint: {"zero_format": "reference"}`).

A gloo world of 2 trains and saves ZeRO-1/2/3 shards under the reference's keys
(`local_sub_partitions_of_fp32_groups` / `single_partition_of_fp32_groups` / `fp32_flat_groups`,
`partition_count`, `param_shapes`).  Checked:

* the files reload through the reference-layout importer into worlds 1 and 4 with exact fp32
  masters and Adam moments;
* a pure-Python re-implementation of the reference's consolidation
  (deepspeed/utils/zero_to_fp32.py:70-151 -- group 0, module order) gives the exact fp32
  weights, and so does this framework's converter;
* several optimizer param groups (weight-decay split) consolidate exactly through the group
  membership the export records; a multi-group file without it is refused, not mis-read.
"""

import glob
import os
from collections import OrderedDict

import pytest
import torch

from common import run_distributed
from simple_model import LinearStack, random_batches

HID = 16


def _net():
    torch.manual_seed(0)
    return LinearStack(input_dim=HID, hidden_dim=24, output_dim=HID, num_layers=3)


def _groups(net, split):
    if not split:
        return net.parameters()
    decay = [p for n, p in net.named_parameters() if n.endswith("weight")]
    other = [p for n, p in net.named_parameters() if not n.endswith("weight")]
    return [{"params": decay}, {"params": other, "weight_decay": 0.0}]


def _conf(stage, fmt, sub_group_size=int(1e12)):
    return {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 1,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-2, "weight_decay": 0.01}},
            "fp16": {"enabled": True, "type": "float32"}, "steps_per_print": 1000,
            "checkpoint": {"zero_format": fmt},
            "zero_optimization": {"stage": stage, "reduce_bucket_size": 200, "allgather_bucket_size": 200,
                                  "stage3_unit_max_numel": 700, "stage3_param_persistence_threshold": 0,
                                  "sub_group_size": sub_group_size}}


def _train_save(root, stage, split, sub_group_size=int(1e12)):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    net = _net()
    eng, *_ = ds.initialize(model=net, model_parameters=_groups(net, split),
                            config_params=_conf(stage, "native", sub_group_size))
    for x, y in random_batches(3, 4, HID, seed=7 + dist.get_rank()):
        loss = eng(x, y)
        eng.backward(loss)
        eng.step()
    eng.save_checkpoint(os.path.join(root, "native"), tag="t")
    eng._config.checkpoint_zero_format = "reference"
    eng.save_checkpoint(os.path.join(root, "ref"), tag="t")


def _expected(root, net):
    """Full fp32 masters and moments per module parameter from the native shards."""
    from deeperspeed_amd.runtime.zero.layout import shards_to_params
    files = sorted(glob.glob(os.path.join(root, "native", "t", "*_optim_states.pt")))
    sds = [torch.load(f, weights_only=True) for f in files]
    osds = [s["optimizer_state_dict"] for s in sds]
    key = osds[0]["fp32_groups_key"]
    out = {"master": {}, "exp_avg": {}, "exp_avg_sq": {}}
    for gi, sig in enumerate(osds[0]["layout"]):
        names = list(sds[0]["param_shapes"][gi].keys())
        per = {"master": shards_to_params([o[key][gi] for o in osds], sig)}
        for m in ("exp_avg", "exp_avg_sq"):
            per[m] = shards_to_params([o["base_optimizer_state"]["state"][gi][m] for o in osds], sig)
        for k in out:
            for i, n in enumerate(names):
                out[k][n] = per[k][i].float().clone()
    return out


def _reference_zero_to_fp32(folder):
    """Pure-Python re-implementation of deepspeed/utils/zero_to_fp32.py:70-151 (0.3.15):
    param group 0 of every rank, module order, ZeRO-3 partitions of floor(numel/world) +
    padding (exact here: every parameter size is a multiple of the world size)."""
    files = sorted(glob.glob(os.path.join(folder, "*_optim_states.pt")))
    sds = [torch.load(f, weights_only=True) for f in files]
    zero_stage = sds[0]["optimizer_state_dict"]["zero_stage"]
    key = {2: "single_partition_of_fp32_groups", 3: "fp32_flat_groups"}[zero_stage]
    param_shapes = sds[0]["param_shapes"]
    flat_groups = [sd["optimizer_state_dict"][key][0] for sd in sds]
    world = sds[0]["optimizer_state_dict"]["partition_count"]
    if zero_stage == 2:
        full = torch.cat(flat_groups, 0)
    out, offset = OrderedDict(), 0
    for name, shape in param_shapes.items():
        n = shape.numel()
        if zero_stage == 2:
            out[name] = full.narrow(0, offset, n).view(shape)
            offset += n
        else:
            rem = n % world
            pad = (world - rem) if rem else 0
            part = int(n / world)
            out[name] = torch.cat(tuple(flat_groups[i].narrow(0, offset, part) for i in range(world)), 0).view(shape)
            offset += part + pad
    return out


def _reload(root, stage, split, done):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.zero.layout import params_to_shard
    net = _net()
    eng, *_ = ds.initialize(model=net, model_parameters=_groups(net, split), config_params=_conf(stage, "native"))
    path, _ = eng.load_checkpoint(os.path.join(root, "ref"), tag="t")
    assert path is not None
    exp = torch.load(os.path.join(root, "expected.pt"), weights_only=True)
    names = {id(p): n for n, p in net.named_parameters()}
    opt = eng.optimizer
    for g in opt.groups:
        want = params_to_shard({i: exp["master"][names[id(p)]] for i, p in enumerate(g.params)}, g, opt.dp_rank,
                               torch.float32)
        assert torch.equal(opt.master_fp32(g).float(), want), "master"
        st = opt.optimizer.state[g.master]
        for m in ("exp_avg", "exp_avg_sq"):
            w = params_to_shard({i: exp[m][names[id(p)]] for i, p in enumerate(g.params)}, g, opt.dp_rank,
                                torch.float32)
            assert torch.equal(st[m].float().cpu(), w), m
        assert int(st["step"]) == 3
    if dist.get_rank() == 0:
        torch.save({"ok": True}, os.path.join(root, done))


@pytest.mark.parametrize("stage,sub_group_size", [(1, int(1e12)), (2, int(1e12)), (3, int(1e12)), (3, 300)])
def test_reference_format_export_roundtrip(tmp_path, stage, sub_group_size):
    root = str(tmp_path)
    run_distributed(_train_save, 2, root, stage, False, sub_group_size)
    f0 = torch.load(os.path.join(root, "ref", "t", "zero_pp_rank_0_mp_rank_00_optim_states.pt"), weights_only=True)
    osd = f0["optimizer_state_dict"]
    key = {1: "local_sub_partitions_of_fp32_groups", 2: "single_partition_of_fp32_groups", 3: "fp32_flat_groups"}[stage]
    assert key in osd and osd["partition_count"] == 2 and osd["zero_stage"] == stage
    assert "layout" not in osd and "dsa_flat_fp32_shards" not in osd
    assert isinstance(f0["param_shapes"], OrderedDict)
    assert all(isinstance(s, torch.Size) for s in f0["param_shapes"].values())
    exp = _expected(root, _net())
    torch.save(exp, os.path.join(root, "expected.pt"))
    for world in (1, 4):
        run_distributed(_reload, world, root, stage, False, f"ok{world}.pt")
        assert os.path.exists(os.path.join(root, f"ok{world}.pt"))
    from deeperspeed_amd.utils.zero_to_fp32 import convert_zero_chkpt_to_fp32_consolid_state_dict
    ours = convert_zero_chkpt_to_fp32_consolid_state_dict(os.path.join(root, "ref", "t"), os.path.join(root, "o.pt"))
    for n, t in exp["master"].items():
        assert torch.equal(ours[n].reshape(-1), t), n
    if stage == 3:
        assert (len(osd["fp32_flat_groups"]) > 1) == (sub_group_size < 1e12)
    if stage in (2, 3) and sub_group_size >= 1e12:  # the reference script reads sub-group 0 only
        ref = _reference_zero_to_fp32(os.path.join(root, "ref", "t"))
        assert list(ref.keys()) == [n for n, _ in _net().named_parameters()]
        for n, t in exp["master"].items():
            assert torch.equal(ref[n].reshape(-1), t), n


@pytest.mark.parametrize("stage", [2, 3])
def test_multi_group_reference_export_consolidates(tmp_path, stage):
    """Weight-decay split: group order (weights, then biases) differs from module order."""
    root = str(tmp_path)
    run_distributed(_train_save, 2, root, stage, True)
    exp = _expected(root, _net())
    torch.save(exp, os.path.join(root, "expected.pt"))
    from deeperspeed_amd.utils.zero_to_fp32 import convert_zero_chkpt_to_fp32_consolid_state_dict
    ours = convert_zero_chkpt_to_fp32_consolid_state_dict(os.path.join(root, "ref", "t"), os.path.join(root, "o.pt"))
    assert list(ours.keys()) == [n for n, _ in _net().named_parameters()]  # module order
    for n, t in exp["master"].items():
        assert torch.equal(ours[n].reshape(-1), t), n
    run_distributed(_reload, 1, root, stage, True, "ok1.pt")
    assert os.path.exists(os.path.join(root, "ok1.pt"))
    # without the recorded membership, several groups cannot be mapped onto module order
    for f in glob.glob(os.path.join(root, "ref", "t", "*_optim_states.pt")):
        sd = torch.load(f, weights_only=True)
        sd.pop("dsa_group_param_names")
        torch.save(sd, f)
    with pytest.raises(ValueError, match="param groups"):
        convert_zero_chkpt_to_fp32_consolid_state_dict(os.path.join(root, "ref", "t"), os.path.join(root, "x.pt"))
