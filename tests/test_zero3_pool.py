"""ZeRO-3 gather window and buffer pool (runtime/zero/stage3.py):

* the prefetch window is bounded by stage3_prefetch_bucket_size (units already in flight
  count against it, so the frontier cannot run away and gather the whole model);
* gathered buffers go back to the persistent pool only when nothing else references them:
  a model whose autograd graph saves a non-leaf VIEW of a weight (``x @ w.t()``) must train
  exactly like the bypass even though the unit is released and its buffer reused before
  backward;
* the pool stops growing after the first step (buffers are reused, no per-unit allocation).
"""

import os

import torch
import torch.nn as nn

from common import run_distributed


class VLin(nn.Module):
    """y = x @ W.t(): matmul saves the non-leaf view W.t() for backward."""

    def __init__(self, d):
        super().__init__()
        self.w = nn.Parameter(torch.randn(d, d) * 0.1)

    def forward(self, x):
        return torch.tanh(torch.matmul(x, self.w.t()))


class ViewNet(nn.Module):
    def __init__(self, d=32, n=4):
        super().__init__()
        self.ls = nn.ModuleList([VLin(d) for _ in range(n)])
        self.out = nn.Linear(d, 1)

    def forward(self, x, y):
        for lin in self.ls:
            x = lin(x)
        return ((self.out(x).squeeze(-1) - y) ** 2).mean()


class Blocks(nn.Module):
    def __init__(self, d=32, n=6):
        super().__init__()
        self.blocks = nn.ModuleList([nn.Sequential(nn.Linear(d, d), nn.Tanh()) for _ in range(n)])
        self.head = nn.Linear(d, 1)

    def forward(self, x, y):
        for b in self.blocks:
            x = b(x)
        return ((self.head(x).squeeze(-1) - y) ** 2).mean()


def _cfg(zero):
    return {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 2,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-2}}, "fp16": {"enabled": True, "type": "bfloat16"}, "fp32_allreduce": False,
            "zero_allow_untested_optimizer": True, "zero_optimization": zero}


def _run(out, tag, net_cls, zero, steps=3):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    torch.manual_seed(3)
    net = net_cls().to(torch.bfloat16)
    eng, *_ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=_cfg(zero))
    g = torch.Generator().manual_seed(11)
    losses, held, live = [], [], []
    opt = eng.optimizer
    for _ in range(steps * 2):
        x, y = torch.randn(4, 32, generator=g).bfloat16(), torch.randn(4, generator=g).bfloat16()
        loss = eng(x, y)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
        if hasattr(opt, "_pool"):
            held.append(opt._pool.held)
    sd = opt.gathered_state_dict(eng.module) if hasattr(opt, "gathered_state_dict") else \
        {k: v.detach().clone() for k, v in eng.module.state_dict().items()}
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "sd": sd, "held": held, "skipped": getattr(opt, "pool_skipped", 0)},
                   os.path.join(out, f"{tag}.pt"))


def test_pooled_buffers_with_saved_weight_views(tmp_path):
    base = {"stage": 3, "stage3_param_persistence_threshold": 0, "stage3_unit_max_numel": 1100,
            "stage3_prefetch_bucket_size": 2000}
    run_distributed(_run, 1, str(tmp_path), "bypass", ViewNet, dict(base))
    run_distributed(_run, 1, str(tmp_path), "sharded", ViewNet, dict(base, stage3_force_sharded=True, grad_accum_dtype="param"))
    a = torch.load(tmp_path / "bypass.pt", weights_only=True)
    b = torch.load(tmp_path / "sharded.pt", weights_only=True)
    assert a["losses"] == b["losses"]
    for k in a["sd"]:
        assert torch.equal(a["sd"][k], b["sd"][k]), k
    assert b["held"][-1] == b["held"][1], "pool kept growing after the first step"
    assert b["skipped"] > 0, "the saved W.t() views should have kept their buffers out of the pool"


def _window(out):
    import deeperspeed_amd as ds
    torch.manual_seed(5)
    net = Blocks().to(torch.bfloat16)
    zero = {"stage": 3, "stage3_force_sharded": True, "stage3_param_persistence_threshold": 0,
            "stage3_unit_max_numel": 1100, "stage3_prefetch_bucket_size": 2200, "stage3_max_live_parameters": 0}
    eng, *_ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=_cfg(zero))
    opt = eng.optimizer
    unit = max(u.numel for u in opt._units)
    peak = [0]
    orig = opt._fetch

    def fetch(u):
        orig(u)
        peak[0] = max(peak[0], opt._live_numel)
    opt._fetch = fetch
    for _ in range(3):
        x, y = torch.randn(4, 32).bfloat16(), torch.randn(4).bfloat16()
        loss = eng(x, y)
        eng.backward(loss)
        eng.step()
    # current unit + the prefetch window (+ one unit of overshoot at the window edge)
    assert peak[0] <= 2200 + 2 * unit, (peak[0], unit)
    total = sum(u.numel for u in opt._units)
    assert peak[0] < total
    torch.save({"peak": peak[0]}, os.path.join(out, "w.pt"))


def test_prefetch_window_bounded(tmp_path):
    run_distributed(_window, 1, str(tmp_path))
