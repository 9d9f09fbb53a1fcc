"""CPU checks of the whole-step graph helpers (runtime/step_graph.py) and of FusedLamb's device
step counter: the bias-corrected step size formed from a tensor step count equals the host
formula, and persistent gradients keep their storage across zero_grad."""

import math

import torch

from deeperspeed_amd.ops.lamb.fused_lamb import FusedLamb
from deeperspeed_amd.runtime.step_graph import persistent_grads


def test_device_lr_matches_host_bias_correction():
    p = torch.nn.Parameter(torch.zeros(8))
    opt = FusedLamb([p], lr=2e-3, betas=(0.9, 0.999))
    opt.enable_device_step()
    group = opt.param_groups[0]
    for t in range(1, 6):
        lr = opt._device_lr(0, group, torch.device("cpu"))
        want = 2e-3 * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        assert abs(float(lr) - want) < 1e-9 * max(1.0, want) + 1e-12
    assert float(opt.device_step(0)) == 5.0


def test_device_lr_starts_from_the_host_step():
    p = torch.nn.Parameter(torch.zeros(4))
    opt = FusedLamb([p], lr=1e-3)
    opt.state[p]["step"] = 7
    opt.state[p]["exp_avg"] = torch.zeros(4)
    opt.state[p]["exp_avg_sq"] = torch.zeros(4)
    opt.enable_device_step()
    opt._device_lr(0, opt.param_groups[0], torch.device("cpu"))
    assert float(opt.device_step(0)) == 8.0


def test_device_lr_without_bias_correction_is_lr():
    p = torch.nn.Parameter(torch.zeros(4))
    opt = FusedLamb([p], lr=5e-4, bias_correction=False)
    opt.enable_device_step()
    assert abs(float(opt._device_lr(0, opt.param_groups[0], torch.device("cpu"))) - 5e-4) < 1e-6 * 5e-4


def test_persistent_grads_bind_every_trainable_parameter_once():
    m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.LayerNorm(3))
    m[1].bias.requires_grad_(False)
    n = persistent_grads(m.parameters())
    assert n == 3  # weight, bias of the linear, weight of the LayerNorm
    ptrs = {id(p): p.grad.data_ptr() for p in m.parameters() if p.requires_grad}
    assert m[1].bias.grad is None
    assert persistent_grads(m.parameters()) == 0  # already bound
    m(torch.randn(2, 4)).sum().backward()
    for p in m.parameters():
        if p.requires_grad:
            assert p.grad.data_ptr() == ptrs[id(p)]  # accumulated in place
