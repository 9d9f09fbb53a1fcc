"""BASELINE config 1: GPT-2 (125M architecture) ZeRO-1 with DeepSpeedCPUAdam on CPU/gloo
world_size=2 (plumbing), plus ZeRO-3 with the tied LM head (external parameter)."""

import os

import pytest
import torch

from common import run_distributed


def _body(out_dir, stage, offload, layers):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt2 import GPT2, get_gpt2_config
    torch.manual_seed(0)
    cfg = get_gpt2_config("gpt2-125m", num_layers=layers, n_positions=128)
    model = GPT2(cfg, dtype=torch.bfloat16)
    zero = {"stage": stage, "reduce_bucket_size": int(2e7), "stage3_unit_max_numel": int(1e7)}
    if offload:
        zero["offload_optimizer"] = {"device": "cpu", "states": "all"}
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 1,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "fp32_allreduce": False, "zero_optimization": zero}
    engine, opt, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    if offload:
        assert type(opt.optimizer).__name__ == "DeepSpeedCPUAdam"
    g = torch.Generator().manual_seed(1 + dist.get_rank())
    ids = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    losses = []
    for _ in range(4):
        loss = engine(ids, labels=ids)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.detach()))
    if dist.get_rank() == 0:
        torch.save(losses, os.path.join(out_dir, f"s{stage}_{offload}.pt"))


@pytest.mark.parametrize("stage,offload", [(1, True), (3, False)])
def test_gpt2_zero_trains(tmp_path, stage, offload):
    run_distributed(_body, 2, str(tmp_path), stage, offload, 2, timeout=600)
    run_distributed(_body, 2, str(tmp_path), 0, False, 2, timeout=600)
    a = torch.load(tmp_path / f"s{stage}_{offload}.pt")
    b = torch.load(tmp_path / "s0_False.pt")
    assert a[-1] < a[0]
    for x, y in zip(a, b):
        assert abs(x - y) < 3e-2 * max(1.0, abs(y)), (a, b)
