"""xGMI bucket sizing ("auto" ZeRO bucket keys)."""

import pytest
import torch

from common import run_distributed
from deeperspeed_amd.runtime.comm import bucket_sizing as bs


def test_auto_bucket_model():
    # bigger rings need bigger buckets to amortise the per-step latency, within the clamps
    sizes = [bs.auto_bucket_elems(n) for n in (2, 4, 8, 16)]
    assert sizes == sorted(sizes) and sizes[0] < sizes[-1]
    assert all(bs.MIN_ELEMS <= v <= bs.MAX_ELEMS for v in sizes)
    assert bs.auto_bucket_elems(1) == bs.MAX_ELEMS
    # at the chosen size the latency term is within the overhead budget of the bandwidth term
    n = 8
    b = bs.auto_bucket_elems(n) * 2
    lat = 2 * (n - 1) * bs.DEFAULT_ALPHA_S
    bw = bs.ring_time_s(b, n) - lat
    assert lat <= bs.DEFAULT_OVERHEAD * bw * 1.001
    assert bs.resolve(12345, 8) == 12345 and bs.resolve("2e6", 8) == 2000000
    assert bs.resolve("auto", 8) == bs.auto_bucket_elems(8)


def _engine_auto(stage):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    world = dist.get_world_size()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
           "fp16": {"enabled": True, "type": "bfloat16"},
           "zero_optimization": {"stage": stage, "reduce_bucket_size": "auto", "allgather_bucket_size": "auto",
                                 "stage3_prefetch_bucket_size": "auto"}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    zc = engine._config.zero_config
    assert zc.reduce_bucket_size == bs.auto_bucket_elems(world)
    assert isinstance(zc.stage3_prefetch_bucket_size, int)
    x = torch.randn(2, 32, dtype=torch.bfloat16)
    loss = engine(x).float().pow(2).mean()
    engine.backward(loss)
    engine.step()


@pytest.mark.parametrize("stage", [0, 2, 3])
def test_engine_accepts_auto_buckets(stage):
    run_distributed(_engine_auto, 2, stage)
