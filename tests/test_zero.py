"""ZeRO stages 0-3 on 2 ranks (gloo/CPU): every stage must train to the same weights.

Reference analogue: tests/unit/test_fp16.py / test_zero.py (ZeRO x offload matrices) -- here
the check is numerical equivalence of the flat-arena ZeRO implementations with plain data
parallelism, plus gradient-accumulation and offload variants.
"""

import os

import pytest
import torch

from common import distributed_test, run_distributed
from simple_model import SimpleModel, base_config, random_batches


def _train_and_dump(out_dir, stage, ga, offload, steps=3, hidden=32, dtype="bfloat16"):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    torch.manual_seed(42)
    model = SimpleModel(hidden)
    zero = {"reduce_bucket_size": 500, "stage3_unit_max_numel": 600, "stage3_param_persistence_threshold": 10}
    if offload == "compact":
        zero["compact_master"] = True
    elif offload == "nvme":
        zero["offload_optimizer"] = {"device": "nvme", "nvme_path": os.path.join(out_dir, "nvme"), "states": "all"}
    elif offload in ("param_cpu", "param_nvme"):
        zero["offload_optimizer"] = {"device": "cpu", "states": "all"}
        zero["offload_param"] = {"device": offload.split("_")[1], "nvme_path": os.path.join(out_dir, "pnvme")}
    elif offload in ("retain", "noretain"):
        zero["stage3_max_live_parameters"] = 10**9 if offload == "retain" else 0
        zero["stage3_max_reuse_distance"] = 10**9 if offload == "retain" else 0
    elif offload:
        zero["offload_optimizer"] = {"device": "cpu", "states": offload}
    cfg = base_config(stage=stage, mb=4, ga=ga, dtype=dtype, **zero)
    if dtype == "float32":
        cfg["optimizer"]["params"]["eps"] = 1e-3  # well-conditioned Adam (test_zero_fp32_exact.py)
    xdt = torch.float32 if dtype == "float32" else torch.bfloat16
    if stage == 0:
        cfg.pop("zero_optimization", None)
    engine, opt, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    rank = dist.get_rank()
    data = random_batches(steps * ga, 4, hidden, seed=100 + rank)
    k = 0
    for _ in range(steps):
        for _ in range(ga):
            x, y = data[k]
            k += 1
            loss = engine(x.to(xdt), y)
            engine.backward(loss)
            engine.step()
    if stage == 3:
        sd = engine.optimizer.gathered_state_dict(engine.module)
    else:
        sd = {k: v.detach().cpu().clone() for k, v in engine.module.state_dict().items()}
    masters = torch.cat([engine.optimizer.master_fp32(g).float() for g in engine.optimizer.groups]) \
        if hasattr(engine.optimizer, "groups") else None
    gathered = getattr(engine.optimizer, "gathered_numel", 0)
    if rank == 0:
        torch.save({"sd": sd, "loss": float(loss), "masters": masters, "gathered": gathered},
                   os.path.join(out_dir, f"s{stage}_ga{ga}_{offload}{'_fp32' if dtype == 'float32' else ''}.pt"))


@pytest.mark.parametrize("ga", [1, 2])
def test_zero_stages_agree(tmp_path, ga):
    """fp32: every stage equals plain data parallelism to fp32 rounding."""
    results = {}
    for stage in (0, 1, 2, 3):
        run_distributed(_train_and_dump, 2, str(tmp_path), stage, ga, None, dtype="float32")
        results[stage] = torch.load(os.path.join(tmp_path, f"s{stage}_ga{ga}_None_fp32.pt"), weights_only=True)
    ref = results[0]["sd"]
    for stage in (1, 2, 3):
        sd = results[stage]["sd"]
        for k in ref:
            assert (ref[k].float() - sd[k].float()).abs().max() <= 1e-6, (stage, k)


def test_zero_stages_agree_bf16(tmp_path):
    """bf16 (the production dtype): the stages differ only by where bf16 gradients are rounded
    and summed; weights stay within a bf16 ulp plus the Adam steps' rounding."""
    results = {}
    for stage in (0, 3):
        run_distributed(_train_and_dump, 2, str(tmp_path), stage, 1, None)
        results[stage] = torch.load(os.path.join(tmp_path, f"s{stage}_ga1_None.pt"), weights_only=True)
    for k in results[0]["sd"]:
        a, b = results[0]["sd"][k].float(), results[3]["sd"][k].float()
        assert torch.allclose(a, b, atol=2e-2, rtol=2e-2), k


def test_zero_offload_matches(tmp_path):
    """ZeRO-Offload (host AVX Adam) equals the on-device fused Adam to fp32 rounding."""
    run_distributed(_train_and_dump, 2, str(tmp_path), 2, 1, None, dtype="float32")
    run_distributed(_train_and_dump, 2, str(tmp_path), 2, 1, "all", dtype="float32")
    run_distributed(_train_and_dump, 2, str(tmp_path), 3, 1, "all", dtype="float32")
    a = torch.load(os.path.join(tmp_path, "s2_ga1_None_fp32.pt"), weights_only=True)["sd"]
    b = torch.load(os.path.join(tmp_path, "s2_ga1_all_fp32.pt"), weights_only=True)["sd"]
    c = torch.load(os.path.join(tmp_path, "s3_ga1_all_fp32.pt"), weights_only=True)["sd"]
    for k in a:
        assert (a[k].float() - b[k].float()).abs().max() <= 1e-6, k
        assert (a[k].float() - c[k].float()).abs().max() <= 1e-6, k


def _single_vs_flat(stage):
    from common import ds_env_single
    ds_env_single()
    import deeperspeed_amd as ds
    torch.manual_seed(0)
    model = SimpleModel(16)
    cfg = base_config(stage=stage, mb=2)
    if stage == 0:
        cfg.pop("zero_optimization", None)
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    for x, y in random_batches(3, 2, 16):
        loss = engine(x.to(torch.bfloat16), y)
        engine.backward(loss)
        engine.step()
    return float(loss)


def test_layout_roundtrip():
    """shards_to_params / params_to_shard invert each other for any world size."""
    from deeperspeed_amd.runtime.zero.layout import (FlatGroup, build_size_buckets, layout_signature,
                                                     params_to_shard, shards_to_params)
    params = [torch.nn.Parameter(torch.randn(n)) for n in (5, 130, 64, 1, 300)]
    for world in (1, 2, 3, 8):
        g = build_size_buckets(FlatGroup(0, 0, torch.float32, False, params), world, 200)
        full = {i: p.detach().reshape(-1).clone() for i, p in enumerate(params)}
        shards = [params_to_shard(full, g, r, torch.float32) for r in range(world)]
        sig = layout_signature([g])[0]
        back = shards_to_params(shards, sig)
        for i, p in enumerate(params):
            assert torch.equal(back[i], full[i])
        # re-shard to another world size
        for w2 in (1, 4):
            g2 = build_size_buckets(FlatGroup(0, 0, torch.float32, False, params), w2, 150)
            s2 = [params_to_shard(back, g2, r, torch.float32) for r in range(w2)]
            b2 = shards_to_params(s2, layout_signature([g2])[0])
            for i in full:
                assert torch.equal(b2[i], full[i])


@pytest.mark.parametrize("stage", [2, 3])
def test_zero_infinity_nvme_matches_cpu_offload(tmp_path, stage):
    """ZeRO-Infinity: fp32 master + moments swapped to NVMe files through the aio engine must
    train exactly like the host-memory offload."""
    run_distributed(_train_and_dump, 2, str(tmp_path), stage, 2, "all")
    run_distributed(_train_and_dump, 2, str(tmp_path), stage, 2, "nvme")
    a = torch.load(os.path.join(tmp_path, f"s{stage}_ga2_all.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, f"s{stage}_ga2_nvme.pt"), weights_only=True)
    for k in a["sd"]:
        assert torch.equal(a["sd"][k], b["sd"][k]), k
    assert torch.equal(a["masters"], b["masters"])
    assert os.path.isdir(os.path.join(tmp_path, "nvme", f"zero_stage_{stage}"))


def _nvme_ckpt_body(out_dir):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    zero = {"reduce_bucket_size": 500, "stage3_unit_max_numel": 600, "stage3_param_persistence_threshold": 10,
            "offload_optimizer": {"device": "nvme", "nvme_path": os.path.join(out_dir, f"nv{dist.get_rank()}"),
                                  "states": "all"}}
    cfg = base_config(stage=3, mb=4, ga=1, **zero)

    def build(seed):
        torch.manual_seed(seed)
        m = SimpleModel(32)
        return ds.initialize(model=m, model_parameters=m.parameters(), config_params=cfg)[0]

    e1 = build(1)
    for x, y in random_batches(3, 4, 32, seed=9 + dist.get_rank()):
        loss = e1(x.to(torch.bfloat16), y)
        e1.backward(loss)
        e1.step()
    e1.save_checkpoint(out_dir, tag="t")
    e2 = build(2)
    e2.load_checkpoint(out_dir, tag="t")
    for g1, g2 in zip(e1.optimizer.groups, e2.optimizer.groups):
        assert torch.equal(e1.optimizer.master_fp32(g1), e2.optimizer.master_fp32(g2))
        assert torch.equal(g1.shard_param, g2.shard_param)
    for gi in range(len(e1.optimizer.groups)):
        assert torch.equal(e1.optimizer._nvme_read_group(gi, "exp_avg_sq"),
                           e2.optimizer._nvme_read_group(gi, "exp_avg_sq"))


def test_nvme_checkpoint_roundtrip(tmp_path):
    run_distributed(_nvme_ckpt_body, 2, str(tmp_path))


@pytest.mark.parametrize("dev", ["cpu", "nvme"])
def test_zero3_param_offload_matches(tmp_path, dev):
    """ZeRO-Infinity parameter offload (bf16 shards in host memory / a file-backed NVMe
    mapping, staged to the device per unit) trains exactly like on-device shards."""
    run_distributed(_train_and_dump, 2, str(tmp_path), 3, 2, "all")
    run_distributed(_train_and_dump, 2, str(tmp_path), 3, 2, f"param_{dev}")
    a = torch.load(os.path.join(tmp_path, "s3_ga2_all.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, f"s3_ga2_param_{dev}.pt"), weights_only=True)
    for k in a["sd"]:
        assert torch.equal(a["sd"][k], b["sd"][k]), k
    assert torch.equal(a["masters"], b["masters"])


def test_zero3_param_retention(tmp_path):
    """stage3_max_live_parameters / stage3_max_reuse_distance: keeping gathered units resident
    across forward->backward and across micro-batches must not change the math, and must cut
    the all-gather volume."""
    run_distributed(_train_and_dump, 2, str(tmp_path), 3, 2, "noretain")
    run_distributed(_train_and_dump, 2, str(tmp_path), 3, 2, "retain")
    a = torch.load(os.path.join(tmp_path, "s3_ga2_noretain.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, "s3_ga2_retain.pt"), weights_only=True)
    for k in a["sd"]:
        assert torch.equal(a["sd"][k], b["sd"][k]), k
    assert torch.equal(a["masters"], b["masters"])
    assert b["gathered"] < 0.6 * a["gathered"], (a["gathered"], b["gathered"])


def test_reuse_distance_table():
    """Reuse distances are measured in parameter elements between uses, cyclic over
    forward + backward of one micro-batch (reference stage3.py PrefetchCoordinator semantics)."""
    from types import SimpleNamespace
    from deeperspeed_amd.runtime.zero.stage3 import DeepSpeedZeroOptimizer_Stage3 as Z3
    z = Z3.__new__(Z3)
    z._units = [SimpleNamespace(numel=n) for n in (10, 20, 30)]
    z._fwd_trace, z._bwd_trace = [0, 1, 2], [2, 1, 0]
    z._compute_reuse()
    assert z._reuse_f == {0: 50 + 30 + 20, 1: 30 + 30, 2: 0}
    assert z._reuse_b == {0: 20 + 10 + 10 + 20, 1: 10 + 10, 2: 0}


def _param_nvme_ckpt_body(out_dir):
    """ZeRO-Infinity parameter partitions on NVMe through the aio swapper: no host copy of the
    shard remains, reads/writes go through the O_DIRECT engine, and a checkpoint round-trips."""
    import torch.distributed as dist
    import deeperspeed_amd as ds
    r = dist.get_rank()
    zero = {"reduce_bucket_size": 500, "stage3_unit_max_numel": 600, "stage3_param_persistence_threshold": 10,
            "offload_optimizer": {"device": "cpu", "states": "all"},
            "offload_param": {"device": "nvme", "nvme_path": os.path.join(out_dir, f"p{r}"), "buffer_count": 3}}
    cfg = base_config(stage=3, mb=4, ga=1, **zero)

    def build(seed):
        torch.manual_seed(seed)
        m = SimpleModel(32)
        return ds.initialize(model=m, model_parameters=m.parameters(), config_params=cfg)[0]

    e1 = build(1)
    sw = e1.optimizer._pswap
    assert sw is not None and all(g.shard_param is None for g in e1.optimizer.groups)
    for x, y in random_batches(3, 4, 32, seed=9 + r):
        loss = e1(x.to(torch.bfloat16), y)
        e1.backward(loss)
        e1.step()
    assert sw.bytes_read > 0 and sw.bytes_written > 0
    files = os.listdir(sw.folder)
    assert files and all(f.endswith(".swp") for f in files)
    e1.save_checkpoint(out_dir, tag="t")
    sd1 = e1.optimizer.gathered_state_dict(e1.module)
    e2 = build(2)
    e2.load_checkpoint(out_dir, tag="t")
    sd2 = e2.optimizer.gathered_state_dict(e2.module)
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k]), k
    for g1, g2 in zip(e1.optimizer.groups, e2.optimizer.groups):
        assert torch.equal(e1.optimizer.param_shard_host(g1), e2.optimizer.param_shard_host(g2))


def test_zero3_param_nvme_aio_checkpoint(tmp_path):
    run_distributed(_param_nvme_ckpt_body, 2, str(tmp_path))
