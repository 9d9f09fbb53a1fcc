"""Loading reference-layout (DeepSpeed 0.3.15 / DeeperSpeed) ZeRO checkpoints.

The shard files are built here in pure Python from the reference's documented partition math
(no reference code is imported or run):
* ZeRO-1: stage1.py:356-401 (sub-partitions of `sub_partition_size`, sub-partition i to rank
  i % dp, comm interval i // dp), saved lean per interval (stage1.py:857-943);
* ZeRO-2: stage2.py:200-250,1150-1168 (flat group padded to a multiple of dp, dp equal
  ranges), padding dropped on the last rank (stage2.py:1687-1745);
* ZeRO-3: partition_parameters.py:547-553,610-690 (each parameter padded to a multiple of dp,
  ceil(numel/dp) per rank), sub-groups by sub_group_size (stage3.py:1332-1356), saved as
  `fp32_flat_groups` + a torch optimizer state dict (stage3.py:3046-3060).
The checkpoint is written for a data-parallel world of 3 and loaded into a world of 2 (gloo):
fp32 masters and Adam moments must come back exactly, re-partitioned into this framework's
own layout; parity with checkpoints produced by the real reference stays unpinned (it ships
none).  Also: this framework's own shards are stored under a key reference tools do not
read, so they fail loudly instead of producing wrong weights.
"""

import os
from collections import OrderedDict

import pytest
import torch

from common import run_distributed
from simple_model import LinearStack, base_config

SAVED_WORLD = 3


def _values(seed, params):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.numel(), generator=g) for p in params]


def _pad(flat, mult):
    r = flat.numel() % mult
    return torch.cat([flat, flat.new_zeros(mult - r)]) if r else flat


def _stage2_files(master, m, v, W):
    flat = [_pad(torch.cat(x), W) for x in (master, m, v)]
    n = sum(t.numel() for t in master)
    ps = flat[0].numel() // W
    out = []
    for r in range(W):
        lo, hi = r * ps, min((r + 1) * ps, n)  # padding dropped (only the last rank has any)
        out.append({"zero_stage": 2, "partition_count": W, "loss_scaler": {"cur_scale": 1.0},
                    "dynamic_loss_scale": False, "overflow": False,
                    "single_partition_of_fp32_groups": [flat[0][lo:hi].clone()],
                    "base_optimizer_state": [{"step": 5, "exp_avg": flat[1][lo:hi].clone(),
                                              "exp_avg_sq": flat[2][lo:hi].clone()}]})
    return out


def _stage1_files(master, m, v, W, sub=40):
    n = sum(t.numel() for t in master)
    flat = [_pad(torch.cat(x), sub * W) for x in (master, m, v)]
    nsub = flat[0].numel() // sub
    out = [{"zero_stage": 1, "partition_count": W, "loss_scaler": {"cur_scale": 1.0}, "dynamic_loss_scale": False,
            "overflow": False, "num_comm_intervals_per_group": [nsub // W],
            "local_sub_partitions_of_fp32_groups": [[]], "base_optimizer_state": [[]]} for _ in range(W)]
    for i in range(nsub):
        r = i % W
        lo, hi = i * sub, min((i + 1) * sub, n)
        hi = max(lo, hi)
        out[r]["local_sub_partitions_of_fp32_groups"][0].append(flat[0][lo:hi].clone())
        out[r]["base_optimizer_state"][0].append({"step": 5, "exp_avg": flat[1][lo:hi].clone(),
                                                  "exp_avg_sq": flat[2][lo:hi].clone()})
    return out


def _stage3_files(master, m, v, W, sub_group_size=300):
    part = [-(-t.numel() // W) for t in master]
    groups, cur, acc = [], [], 0
    for j, ps in enumerate(part):
        cur.append(j)
        acc += ps
        if acc >= sub_group_size or j == len(part) - 1:
            groups.append(cur)
            cur, acc = [], 0
    out = []
    for r in range(W):
        def rank_flat(ts, members):
            return torch.cat([_pad(ts[j], W)[r * part[j]:(r + 1) * part[j]] for j in members])
        flats = [rank_flat(master, grp) for grp in groups]
        state = {k: {"step": 5, "exp_avg": rank_flat(m, grp), "exp_avg_sq": rank_flat(v, grp)}
                 for k, grp in enumerate(groups)}
        out.append({"zero_stage": 3, "partition_count": W, "loss_scaler": {"cur_scale": 1.0},
                    "dynamic_loss_scale": False, "overflow": False, "fp32_flat_groups": flats,
                    "optimizer_state_dict": {"state": state,
                                             "param_groups": [{"lr": 1e-2, "params": list(range(len(groups)))}]}})
    assert len(groups) > 1  # several sub-groups exercised
    return out


def _write(ckpt, stage, net):
    params = [p for p in net.parameters()]
    master, m, v = _values(1, params), _values(2, params), _values(3, params)
    m = [x.abs() * 0.1 for x in m]
    v = [x.abs() * 0.01 for x in v]
    tag = os.path.join(ckpt, "global_step5")
    os.makedirs(tag, exist_ok=True)
    files = {1: _stage1_files, 2: _stage2_files, 3: _stage3_files}[stage](master, m, v, SAVED_WORLD)
    shapes = OrderedDict((n, p.shape) for n, p in net.named_parameters())
    for r, osd in enumerate(files):
        torch.save({"optimizer_state_dict": osd, "param_shapes": shapes},
                   os.path.join(tag, f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt"))
    module = {} if stage == 3 else {n: t.view(p.shape).to(torch.bfloat16)
                                    for (n, p), t in zip(net.named_parameters(), master)}
    # ZeRO-3 model states are written per data-parallel rank (reference engine.py _get_ckpt_name)
    names = [f"zero_pp_rank_{r}_mp_rank_00_model_states.pt" for r in range(SAVED_WORLD)] if stage == 3 \
        else ["mp_rank_00_model_states.pt"]
    for name in names:
        torch.save({"module": module, "optimizer": None, "lr_scheduler": None, "csr_tensor_module_names": set(),
                    "skipped_steps": 0, "global_steps": 5, "global_samples": 40, "dp_world_size": SAVED_WORLD,
                    "mp_world_size": 1}, os.path.join(tag, name))
    with open(os.path.join(ckpt, "latest"), "w") as f:
        f.write("global_step5")
    return master, m, v


def _load(ckpt, stage, out):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.zero.layout import params_to_shard
    torch.manual_seed(0)
    net = LinearStack(input_dim=16, hidden_dim=24, output_dim=16, num_layers=3).to(torch.bfloat16)
    if dist.get_rank() == 0:
        _write(ckpt, stage, net)
    dist.barrier()
    params = list(net.parameters())
    master, m, v = _values(1, params), _values(2, params), _values(3, params)
    m = [x.abs() * 0.1 for x in m]
    v = [x.abs() * 0.01 for x in v]
    eng, *_ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=base_config(stage=stage))
    path, _ = eng.load_checkpoint(ckpt)
    assert path is not None and eng.global_steps == 5
    opt = eng.optimizer
    pos = {id(p): j for j, p in enumerate(params)}
    for g in opt.groups:
        idx = {i: pos[id(p)] for i, p in enumerate(g.params)}
        want = params_to_shard({i: master[j] for i, j in idx.items()}, g, opt.dp_rank, torch.float32)
        assert torch.equal(opt.master_fp32(g).float(), want), "fp32 master"
        st = opt.optimizer.state[g.master]
        for name, ref in (("exp_avg", m), ("exp_avg_sq", v)):
            w = params_to_shard({i: ref[j] for i, j in idx.items()}, g, opt.dp_rank, torch.float32)
            assert torch.equal(st[name].float().cpu(), w), name
        assert int(st["step"]) == 5
    full = opt.gathered_state_dict(eng.module) if stage == 3 else eng.module.state_dict()
    for (n, p), t in zip(net.named_parameters(), master):
        assert torch.equal(full[n].float().cpu().reshape(-1), t.to(torch.bfloat16).float()), n
    if dist.get_rank() == 0:
        torch.save({"ok": True}, os.path.join(out, "ok.pt"))


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_load_reference_layout_checkpoint(tmp_path, stage):
    run_distributed(_load, 2, str(tmp_path / "ckpt"), stage, str(tmp_path))
    assert (tmp_path / "ok.pt").exists()


def _save_own(ckpt):
    import deeperspeed_amd as ds
    torch.manual_seed(0)
    net = LinearStack(input_dim=16, hidden_dim=24, output_dim=16, num_layers=3).to(torch.bfloat16)
    eng, *_ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=base_config(stage=2))
    eng.save_checkpoint(ckpt, tag="t")


def test_own_shards_refuse_reference_keys(tmp_path):
    run_distributed(_save_own, 2, str(tmp_path))
    sd = torch.load(tmp_path / "t" / "zero_pp_rank_0_mp_rank_00_optim_states.pt", weights_only=True)
    osd = sd["optimizer_state_dict"]
    assert osd["dsa_layout_version"] >= 2 and "layout" in osd
    # the reference converter reads exactly these keys: they must be absent
    assert "single_partition_of_fp32_groups" not in osd and "fp32_flat_groups" not in osd
    # this framework's converter (copied next to the shards) consolidates them
    from deeperspeed_amd.utils.zero_to_fp32 import convert_zero_chkpt_to_fp32_consolid_state_dict
    out = convert_zero_chkpt_to_fp32_consolid_state_dict(str(tmp_path / "t"), str(tmp_path / "full.pt"))
    assert len(out) == len(list(LinearStack(input_dim=16, hidden_dim=24, output_dim=16, num_layers=3).parameters()))


@pytest.mark.parametrize("stage", [2, 3])
def test_zero_to_fp32_reads_reference_layout(tmp_path, stage):
    from deeperspeed_amd.utils.zero_to_fp32 import convert_zero_chkpt_to_fp32_consolid_state_dict
    torch.manual_seed(0)
    net = LinearStack(input_dim=16, hidden_dim=24, output_dim=16, num_layers=3)
    master, _, _ = _write(str(tmp_path), stage, net)
    out = convert_zero_chkpt_to_fp32_consolid_state_dict(str(tmp_path / "global_step5"), str(tmp_path / "f.pt"))
    for (n, p), t in zip(net.named_parameters(), master):
        assert torch.equal(out[n], t.view(p.shape)), n
