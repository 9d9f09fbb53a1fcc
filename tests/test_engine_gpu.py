"""End-to-end engine runs of the flagship model on one MI355X (ZeRO 0-3, offload modes)."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _run(stage, offload=None, steps=4, ga=2):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("gpt-neox-125m", num_layers=2, max_seq_len=128)
    model = GPTNeoX(cfg, device=dev, dtype=torch.bfloat16)
    z = {"stage": stage, "reduce_bucket_size": int(5e6)}
    if offload:
        z["offload_optimizer"] = {"device": "cpu", "pin_memory": True, "states": offload}
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": ga,
            "optimizer": {"type": "Adam", "params": {"lr": 3e-4}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "fp32_allreduce": False, "gradient_clipping": 1.0, "zero_optimization": z}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ids = torch.randint(0, cfg.vocab_size, (2, 128), device=dev, generator=g)
    losses = []
    for _ in range(steps):
        for _ in range(ga):
            loss = engine(ids, labels=ids)
            engine.backward(loss)
            engine.step()
        losses.append(float(loss))
    return losses


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_engine_loss_decreases(stage):
    losses = _run(stage)
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("offload", ["master", "all"])
def test_engine_offload(offload):
    base = _run(3, None, steps=3, ga=1)
    off = _run(3, offload, steps=3, ga=1)
    assert abs(base[-1] - off[-1]) < 5e-2 * max(1.0, abs(base[-1]))
