"""Checkpoint save/load (reference analogue: tests/unit/test_checkpointing.py): model, optimizer and
LR-scheduler state round trips for ZeRO 0-3, the on-disk layout, `latest`, tag validation, and
elastic restore of ZeRO shards into a different data-parallel world size."""

import os

import pytest
import torch

from common import run_distributed
from simple_model import SimpleModel, base_config, random_batches


def _engine(stage, hidden=32, sched=True, offload=None):
    import deeperspeed_amd as ds
    torch.manual_seed(11)
    model = SimpleModel(hidden)
    z = {"reduce_bucket_size": 400, "stage3_unit_max_numel": 600, "stage3_param_persistence_threshold": 10}
    if offload:
        z["offload_optimizer"] = {"device": "cpu", "states": offload}
    cfg = base_config(stage=stage, mb=2, **z)
    if stage == 0:
        cfg.pop("zero_optimization", None)
    if sched:
        cfg["scheduler"] = {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 0.01,
                                                           "warmup_num_steps": 10}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    return engine


def _train(engine, steps, seed):
    import torch.distributed as dist
    rank = dist.get_rank() if dist.is_initialized() else 0
    for x, y in random_batches(steps, 2, 32, seed=seed + rank):
        loss = engine(x.to(torch.bfloat16), y)
        engine.backward(loss)
        engine.step()
    return float(loss)


def _params(engine):
    if engine.zero_optimization_stage() == 3:
        return engine.optimizer.gathered_state_dict(engine.module)
    return {k: v.detach().cpu().clone() for k, v in engine.module.state_dict().items()}


def _masters(engine):
    return [g.master.detach().cpu().clone() for g in engine.optimizer.groups]


def _save_load_body(save_dir, stage, offload=None):
    import torch.distributed as dist
    e1 = _engine(stage, offload=offload)
    _train(e1, 3, 0)
    e1.save_checkpoint(save_dir, client_state={"extra": 7})
    p1 = _params(e1)
    m1 = _masters(e1)
    lr1 = e1.get_lr()
    # continue training e1 and a freshly loaded e2 in lockstep: they must stay identical
    e2 = _engine(stage, offload=offload)
    path, client = e2.load_checkpoint(save_dir)
    assert path is not None and client["extra"] == 7
    assert e2.global_steps == e1.global_steps == 3
    assert e2.get_lr() == lr1
    p2 = _params(e2)
    for k in p1:
        assert torch.equal(p1[k], p2[k]), k
    for a, b in zip(m1, _masters(e2)):
        assert torch.equal(a, b)
    l1 = _train(e1, 2, 5)
    l2 = _train(e2, 2, 5)
    assert abs(l1 - l2) < 1e-6
    p1, p2 = _params(e1), _params(e2)
    for k in p1:
        assert torch.equal(p1[k], p2[k]), k
    if dist.get_rank() == 0:
        tag = "global_step3"
        assert open(os.path.join(save_dir, "latest")).read().strip() == tag
        files = sorted(os.listdir(os.path.join(save_dir, tag)))
        if stage == 0:
            assert files == ["mp_rank_00_model_states.pt"]
        elif stage in (1, 2):
            assert "mp_rank_00_model_states.pt" in files
            assert "zero_pp_rank_0_mp_rank_00_optim_states.pt" in files
            assert "zero_pp_rank_1_mp_rank_00_optim_states.pt" in files
            assert "zero_to_fp32.py" in files
        else:
            assert "zero_pp_rank_0_mp_rank_00_model_states.pt" in files
            assert "zero_pp_rank_1_mp_rank_00_optim_states.pt" in files


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_checkpoint_roundtrip(tmp_path, stage):
    run_distributed(_save_load_body, 2, str(tmp_path), stage)


def test_checkpoint_roundtrip_offload(tmp_path):
    run_distributed(_save_load_body, 2, str(tmp_path), 2, "all")


def _elastic_save(save_dir, stage):
    e = _engine(stage, sched=False)
    _train(e, 2, 0)
    e.save_checkpoint(save_dir, tag="ckpt")
    import torch.distributed as dist
    if dist.get_rank() == 0:
        torch.save({"masters_rank0": _masters(e), "params": _params(e)}, os.path.join(save_dir, "ref.pt"))
    else:
        torch.save({"masters_rank1": _masters(e)}, os.path.join(save_dir, "ref1.pt"))


def _elastic_load(save_dir, stage):
    e = _engine(stage, sched=False)
    e.load_checkpoint(save_dir, tag="ckpt")
    ref = torch.load(os.path.join(save_dir, "ref.pt"), weights_only=True)
    p = _params(e)
    for k, v in ref["params"].items():
        assert torch.equal(p[k], v), k
    # the whole fp32 master, reconstructed from two shards, must equal the single-rank master
    from deeperspeed_amd.runtime.zero.layout import shards_to_params
    import glob
    sd0 = torch.load(glob.glob(os.path.join(save_dir, "ckpt", "zero_pp_rank_0_*optim_states.pt"))[0],
                     weights_only=True)["optimizer_state_dict"]
    sd1 = torch.load(glob.glob(os.path.join(save_dir, "ckpt", "zero_pp_rank_1_*optim_states.pt"))[0],
                     weights_only=True)["optimizer_state_dict"]
    key = sd0["fp32_groups_key"]
    for gi, g in enumerate(e.optimizer.groups):
        full = shards_to_params([sd0[key][gi], sd1[key][gi]], sd0["layout"][gi])
        mine = shards_to_params([g.master.cpu()], __import__(
            "deeperspeed_amd.runtime.zero.layout", fromlist=["x"]).layout_signature([g])[0])
        for i in full:
            assert torch.equal(full[i], mine[i])
    _train(e, 1, 9)


@pytest.mark.parametrize("stage", [1, 2])
def test_elastic_zero_checkpoint_dp2_to_dp1(tmp_path, stage):
    run_distributed(_elastic_save, 2, str(tmp_path), stage)
    run_distributed(_elastic_load, 1, str(tmp_path), stage)


def _tag_body(save_dir, mode):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    torch.manual_seed(0)
    model = SimpleModel(8)
    cfg = base_config(stage=1, mb=2)
    cfg["checkpoint"] = {"tag_validation": mode}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    tag = f"tag-{dist.get_rank()}"
    if mode == "FAIL":
        with pytest.raises(AssertionError):
            engine.save_checkpoint(save_dir, tag=tag)
    else:
        engine.save_checkpoint(save_dir, tag=tag)


@pytest.mark.parametrize("mode", ["WARN", "IGNORE", "FAIL"])
def test_checkpoint_tag_validation(tmp_path, mode):
    run_distributed(_tag_body, 2, str(tmp_path), mode)


def test_zero_to_fp32(tmp_path):
    run_distributed(_elastic_save, 2, str(tmp_path), 2)
    from deeperspeed_amd.utils.zero_to_fp32 import convert_zero_chkpt_to_fp32_consolid_state_dict
    out = str(tmp_path / "fp32.bin")
    convert_zero_chkpt_to_fp32_consolid_state_dict(os.path.join(str(tmp_path), "ckpt"), out)
    sd = torch.load(out, weights_only=True)
    ref = torch.load(os.path.join(str(tmp_path), "ref.pt"), weights_only=True)["params"]
    for k, v in ref.items():
        assert sd[k].dtype == torch.float32
        assert torch.allclose(sd[k].to(v.dtype).float(), v.float(), atol=1e-2), k


def _fp16_weights_resume_body(save_dir, stage):
    """load_from_fp32_weights=false: the masters must be rebuilt from the loaded bf16 weights
    (reference stage2.py:1877-1880 _restore_from_fp16_weights), so a resumed engine keeps
    training exactly like one restarted from a checkpoint whose masters equal its weights."""
    import deeperspeed_amd as ds
    e1 = _engine(stage, sched=False)
    _train(e1, 3, 0)
    e1.save_checkpoint(save_dir)
    p1 = _params(e1)

    def fresh():
        torch.manual_seed(11)
        model = SimpleModel(32)
        z = {"reduce_bucket_size": 400, "stage3_unit_max_numel": 600, "stage3_param_persistence_threshold": 10,
             "load_from_fp32_weights": False}
        cfg = base_config(stage=stage, mb=2, **z)
        return ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)[0]

    e2 = fresh()
    e2.load_checkpoint(save_dir)
    p2 = _params(e2)
    for k in p1:
        assert torch.equal(p1[k], p2[k]), k
    # masters == bf16 weights (upcast), shard for shard
    for g in e2.optimizer.groups:
        src = e2.optimizer._low_precision_shard(g)
        assert torch.equal(e2.optimizer.master_fp32(g).float(), src.detach().float().cpu())
    _train(e2, 1, 5)
    p3 = _params(e2)
    moved = [k for k in p1 if not torch.equal(p1[k], p3[k])]
    diffs = max((p1[k].float() - p3[k].float()).abs().max().item() for k in p1)
    assert moved and diffs < 0.05, (moved, diffs)  # one Adam step (lr 1e-2) away, not back at init


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_resume_from_fp16_weights(tmp_path, stage):
    run_distributed(_fp16_weights_resume_body, 2, str(tmp_path), stage)
