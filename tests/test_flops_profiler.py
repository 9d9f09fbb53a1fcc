"""FLOPs profiler (reference tests/unit/test_flops_profiler.py)."""

import torch
import torch.nn as nn

from common import run_distributed


def test_flops_profiler_counts_macs():
    from deeperspeed_amd.profiling.flops_profiler import FlopsProfiler, get_model_profile
    model = nn.Sequential(nn.Linear(10, 20), nn.ReLU(), nn.Linear(20, 5))
    prof = FlopsProfiler(model)
    prof.start_profile()
    model(torch.randn(4, 10))
    assert prof.get_total_flops() == 4 * 10 * 20 + 4 * 20 + 4 * 20 * 5
    assert prof.get_total_params() == 10 * 20 + 20 + 20 * 5 + 5
    assert model[0].__flops__ == 800 and model[2].__flops__ == 400
    text = prof.print_model_profile(profile_step=1, detailed=True, output_file=None)
    assert "Detailed Profile" in text and "Linear" in text
    prof.end_profile()
    assert not hasattr(model[0], "__flops__")
    macs, params = get_model_profile(nn.Linear(8, 8), input_res=(3, 8), print_profile=False, as_string=False)
    assert macs == 3 * 8 * 8 and params == 72


def test_flops_profiler_bmm_and_conv():
    from deeperspeed_amd.profiling.flops_profiler import FlopsProfiler

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 4, 3, padding=1)

        def forward(self, x, a, b):
            return self.conv(x).sum() + torch.bmm(a, b).sum()

    m = M()
    prof = FlopsProfiler(m)
    prof.start_profile()
    m(torch.randn(1, 3, 8, 8), torch.randn(2, 3, 5), torch.randn(2, 5, 7))
    conv = 1 * 4 * 8 * 8 * 3 * 3 * 3
    assert m.conv.__flops__ == conv
    assert prof.get_total_flops() >= conv + 2 * 3 * 5 * 7
    prof.end_profile()


def _engine_body():
    import deeperspeed_amd as ds
    from simple_model import SimpleModel, random_batches
    model = SimpleModel(16)
    cfg = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
           "flops_profiler": {"enabled": True, "profile_step": 1, "module_depth": -1, "top_modules": 2,
                              "detailed": True}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    for x, y in random_batches(3, 4, 16):
        loss = engine(x, y)
        engine.backward(loss)
        engine.step()


def test_engine_flops_profiler_step():
    run_distributed(_engine_body, 1)
