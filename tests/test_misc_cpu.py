"""LR schedules, elasticity, native CPU Adam, async I/O, activation checkpointing, PLD, CSR, GNS
(reference analogues: test_lr_schedulers.py, test_elastic.py, test_cpu_adam.py, csrc/aio/py_test,
test_activation_checkpointing.py, test_pld.py, test_csr.py)."""

import math
import os

import pytest
import torch

from deeperspeed_amd.runtime import lr_schedules


def _opt(lr=0.1):
    return torch.optim.SGD([torch.nn.Parameter(torch.zeros(2))], lr=lr, momentum=0.9)


def test_warmup_lr_log_schedule():
    opt = _opt()
    s = lr_schedules.WarmupLR(opt, warmup_min_lr=0.0, warmup_max_lr=0.01, warmup_num_steps=10)
    lrs = []
    for _ in range(15):
        s.step()
        lrs.append(opt.param_groups[0]["lr"])
    assert lrs[0] == 0.0
    assert all(lrs[i] <= lrs[i + 1] + 1e-12 for i in range(14))
    assert abs(lrs[-1] - 0.01) < 1e-12
    assert abs(lrs[4] - 0.01 * math.log(5) / math.log(10)) < 1e-9


def test_warmup_decay_lr():
    opt = _opt()
    s = lr_schedules.WarmupDecayLR(opt, total_num_steps=20, warmup_min_lr=0.0, warmup_max_lr=0.01,
                                   warmup_num_steps=5)
    for _ in range(21):
        s.step()
    assert opt.param_groups[0]["lr"] == 0.0
    sd = s.state_dict()
    s2 = lr_schedules.WarmupDecayLR(_opt(), total_num_steps=20, warmup_max_lr=0.01, warmup_num_steps=5)
    s2.load_state_dict(sd)
    assert s2.last_batch_iteration == s.last_batch_iteration


def test_one_cycle_lr_and_momentum():
    opt = torch.optim.Adam([torch.nn.Parameter(torch.zeros(2))])
    s = lr_schedules.OneCycle(opt, cycle_min_lr=0.01, cycle_max_lr=0.1, cycle_first_step_size=10,
                              cycle_momentum=True, cycle_min_mom=0.8, cycle_max_mom=0.9, decay_lr_rate=0.1,
                              decay_step_size=5)
    lrs, moms = [], []
    for _ in range(30):
        s.step()
        lrs.append(opt.param_groups[0]["lr"])
        moms.append(opt.param_groups[0]["betas"][0])
    peak = max(range(30), key=lambda i: lrs[i])
    assert abs(lrs[peak] - 0.1) < 1e-9 and peak in (9, 10)
    assert abs(moms[peak] - 0.8) < 1e-9  # momentum is inverse to lr
    assert lrs[25] < 0.01  # decays after the cycle


def test_lr_range_test():
    opt = _opt()
    s = lr_schedules.LRRangeTest(opt, lr_range_test_min_lr=1e-3, lr_range_test_step_size=10,
                                 lr_range_test_step_rate=1.0, lr_range_test_staircase=True)
    for _ in range(25):
        s.step()
    assert abs(opt.param_groups[0]["lr"] - 1e-3 * 3) < 1e-12


def test_config_from_args():
    import argparse
    p = lr_schedules.add_tuning_arguments(argparse.ArgumentParser())
    a = p.parse_args(["--lr_schedule", "WarmupLR", "--warmup_num_steps", "7"])
    cfg, err = lr_schedules.get_config_from_args(a)
    assert err is None and cfg["type"] == "WarmupLR" and cfg["params"]["warmup_num_steps"] == 7
    lr, _ = lr_schedules.get_lr_from_config(cfg)
    assert lr == 0.001


def test_elastic_config():
    from deeperspeed_amd.elasticity import compute_elastic_config
    from deeperspeed_amd.elasticity.config import ElasticityIncompatibleWorldSize
    cfg = {"elasticity": {"enabled": True, "max_train_batch_size": 10000, "micro_batch_sizes": [8, 12, 16, 17],
                          "min_gpus": 32, "max_gpus": 1500, "min_time": 20, "version": 0.1}}
    bs, gpus = compute_elastic_config(cfg, "0.3.15")
    assert bs == 9792
    assert len(gpus) == 23
    bs2, gpus2, mb = compute_elastic_config(cfg, "0.3.15", world_size=gpus[0])
    assert bs2 == bs and (bs // gpus[0]) % mb == 0
    with pytest.raises(ElasticityIncompatibleWorldSize):
        compute_elastic_config(cfg, "0.3.15", world_size=7)


def test_cpu_adam_matches_torch():
    from deeperspeed_amd.ops.adam.cpu_adam import DeepSpeedCPUAdam, cpu_ops
    torch.manual_seed(0)
    for n in (64, 1000003):
        p1 = torch.nn.Parameter(torch.randn(n))
        p2 = torch.nn.Parameter(p1.detach().clone())
        o1 = DeepSpeedCPUAdam([p1], lr=1e-2, weight_decay=0.01, adamw_mode=True)
        o2 = torch.optim.AdamW([p2], lr=1e-2, weight_decay=0.01)
        for _ in range(5):
            g = torch.randn(n)
            p1.grad, p2.grad = g.clone(), g.clone()
            o1.step()
            o2.step()
        assert torch.allclose(p1, p2, atol=1e-5, rtol=1e-5)
    assert cpu_ops().adam_isa() in (0, 1, 2)


def test_cpu_adam_bf16_output_and_isa_paths(monkeypatch):
    from deeperspeed_amd.ops.adam.cpu_adam import cpu_ops
    ops = cpu_ops()
    n = 4099
    base = torch.randn(n)
    g = torch.randn(n)
    out = {}
    for isa in ("0", "1"):
        p = base.clone()
        m, v = torch.zeros(n), torch.zeros(n)
        o = torch.empty(n, dtype=torch.bfloat16)
        ops.adam_update(p, g, m, v, 1e-2, 0.9, 0.999, 1e-8, 0.0, 1, True, 1.0, True, o)
        out[isa] = (p, o)
        assert torch.equal(o, p.to(torch.bfloat16))
    assert torch.allclose(out["0"][0], out["1"][0], atol=1e-6)


def test_aio_roundtrip(tmp_path):
    from deeperspeed_amd.ops.aio import AsyncIOBuilder
    aio = AsyncIOBuilder().load()
    h = aio.aio_handle(block_size=1 << 16, queue_depth=8, single_submit=False, overlap_events=True, thread_count=3)
    x = torch.randn(300001)
    f = str(tmp_path / "x.swp")
    assert h.sync_pwrite(x, f) == 1
    y = torch.empty_like(x)
    assert h.sync_pread(y, f) == 1
    assert torch.equal(x, y)
    z = torch.empty_like(x)
    h.async_pread(z, f)
    assert h.wait() == 1 and torch.equal(x, z)
    w = torch.empty_like(x)
    aio.deepspeed_memcpy(w, x)
    assert torch.equal(w, x)


def test_activation_checkpoint_equivalence():
    from deeperspeed_amd.runtime.activation_checkpointing import checkpointing
    torch.manual_seed(1)
    layer = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Dropout(0.3),
                                torch.nn.Linear(32, 16))
    x = torch.randn(4, 16, requires_grad=True)
    torch.manual_seed(5)
    y1 = checkpointing.checkpoint(layer, x)
    y1.sum().backward()
    g1 = [p.grad.clone() for p in layer.parameters()]
    gx1 = x.grad.clone()
    for p in layer.parameters():
        p.grad = None
    x.grad = None
    torch.manual_seed(5)
    y2 = layer(x)
    y2.sum().backward()
    assert torch.allclose(y1, y2)
    assert torch.allclose(gx1, x.grad)
    for a, p in zip(g1, layer.parameters()):
        assert torch.allclose(a, p.grad)


def test_activation_checkpoint_non_tensor_args():
    from deeperspeed_amd.runtime.activation_checkpointing import checkpointing

    def f(x, scale, flag):
        return x * scale if flag else x

    x = torch.randn(3, requires_grad=True)
    y = checkpointing.checkpoint(f, x, 2.0, True)
    y.sum().backward()
    assert torch.allclose(x.grad, torch.full((3,), 2.0))


def test_pld_theta():
    from deeperspeed_amd.runtime.progressive_layer_drop import ProgressiveLayerDrop
    pld = ProgressiveLayerDrop(theta=0.5, gamma=0.1)
    pld.update_state(0)
    assert pld.get_theta() == 1.0
    pld.update_state(10)
    assert abs(pld.get_theta() - (0.5 * math.exp(-1.0) + 0.5)) < 1e-12
    assert pld.get_state() == {"progressive_layer_drop": True, "pld_theta": pld.get_theta()}


def test_csr_tensor():
    from deeperspeed_amd.runtime.csr_tensor import CSRTensor
    d = torch.zeros(10, 4)
    d[2] = 1.0
    d[7] = torch.arange(4.0)
    c = CSRTensor(d)
    assert c.indices.tolist() == [2, 7]
    assert torch.equal(c.to_dense(), d)
    c.add(CSRTensor(d))
    assert torch.equal(c.to_dense(), 2 * d)


def test_gradient_noise_scale():
    from deeperspeed_amd.runtime.utils import GradientNoiseScale
    m = torch.nn.Linear(4, 4)
    gns = GradientNoiseScale(m, batch_size_small=4, n_batches=2, beta=0.9)
    for i in range(4):
        m.weight.grad = torch.randn(4, 4)
        m.bias.grad = torch.randn(4)
        gns.update()
    assert gns.noise_scale is not None and gns.n_updates == 4


def test_batch_size_scheduler():
    """bs_schedules.BatchSizeScheduler: truncated linear ramp, merged duplicate intervals,
    stepwise lookup (reference bs_schedules.py:28-56)."""
    from deeperspeed_amd.runtime.bs_schedules import BatchSizeScheduler
    s = BatchSizeScheduler(final_batch_size=16, num_intervals=8, warmup_num_steps=10000)
    assert s.schedule == {0: 1, 1428: 3, 2857: 5, 4285: 7, 5714: 9, 7142: 11, 8571: 13, 10000: 16}
    seen = []
    for _ in range(10002):
        s.step()
        if not seen or seen[-1][1] != s.current_batch_size:
            seen.append((s.last_batch_iteration, s.current_batch_size))
    assert seen == [(0, 1), (1428, 3), (2857, 5), (4285, 7), (5714, 9), (7142, 11), (8571, 13), (10000, 16)]
    # duplicates merge: sizes 2,2,2,3 -> two intervals
    d = BatchSizeScheduler(final_batch_size=3, min_batch_size_multiplier=0.5, warmup_num_steps=30, num_intervals=4)
    assert d.schedule == {0: 2, 30: 3}
    d.load_state_dict({"last_batch_iteration": 29})
    d.step()
    assert d.current_batch_size == 3 and d.state_dict() == {"last_batch_iteration": 30}


def test_pipe_visualizer():
    from deeperspeed_amd.runtime.pipe.pipe_visualizer import pipeline_visualizer, schedule_grid
    grid = schedule_grid(4, 4)
    for row in grid:  # every stage runs each micro-batch forward and backward once
        cells = " / ".join(row)
        assert cells.count("fwd") == 4 and cells.count("bwd") == 4
    out = pipeline_visualizer(4, 4)
    assert "GPU 3" in out and "Idle Time: 24" in out and "Non Idle Time: 32" in out
    assert "reduce_grads" in pipeline_visualizer(2, 2, include_all=True)
