"""Asynchronous pipeline p2p (gloo; the same engine code drives RCCL send/recv): sends stay in
flight across the following compute instruction, receives are posted ahead of the compute
before them and waited only by their consumer -- with losses and weights identical to the
blocking transfers (DSA_PIPE_ASYNC_P2P=0), for PP=2 and PP=4, bf16 with fp32 communication.
Reference: deepspeed/runtime/pipe/engine.py:939-1070 (blocking) and p2p.py:31-61."""

import os

import pytest
import torch
import torch.nn as nn

from common import run_distributed

HID = 16


def _body(out_dir, stages, async_p2p, fp32_comm):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.pipe.module import LayerSpec, PipelineModule
    os.environ["DSA_PIPE_ASYNC_P2P"] = "1" if async_p2p else "0"
    torch.manual_seed(0)
    specs = []
    for _ in range(2 * stages):
        specs += [LayerSpec(nn.Linear, HID, HID), LayerSpec(nn.ReLU)]
    model = PipelineModule(layers=specs, num_stages=stages, loss_fn=nn.CrossEntropyLoss(),
                           partition_method="uniform", seed_layers=True, base_seed=3)
    cfg = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 6,
           "optimizer": {"type": "Adam", "params": {"lr": 1e-2}}, "steps_per_print": 1000,
           "fp16": {"enabled": True, "type": "bfloat16"}, "fp32_allreduce": fp32_comm}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=list(model.parameters()), config_params=cfg)
    engine.p2p_trace = []
    g = torch.Generator().manual_seed(5)
    data = [(torch.randn(4, HID, generator=g).to(torch.bfloat16), torch.randint(0, HID, (4,), generator=g))
            for _ in range(6)]
    losses = [float(engine.train_batch(iter(data))) for _ in range(3)]
    sd = {f"{k}": v.float().clone() for k, v in engine.module.state_dict().items()}
    res = {"losses": losses, "sd": sd, "trace": engine.p2p_trace}
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, res)
    if dist.get_rank() == 0:
        torch.save(gathered, os.path.join(out_dir, f"s{stages}_a{int(async_p2p)}_f{int(fp32_comm)}.pt"))


@pytest.mark.parametrize("stages,fp32_comm", [(2, False), (4, True)])
def test_async_p2p_matches_blocking(tmp_path, stages, fp32_comm):
    run_distributed(_body, stages, str(tmp_path), stages, False, fp32_comm)
    run_distributed(_body, stages, str(tmp_path), stages, True, fp32_comm)
    sync = torch.load(tmp_path / f"s{stages}_a0_f{int(fp32_comm)}.pt", weights_only=False)
    asyn = torch.load(tmp_path / f"s{stages}_a1_f{int(fp32_comm)}.pt", weights_only=False)
    for a, b in zip(sync, asyn):
        assert a["losses"] == b["losses"]
        for k in a["sd"]:
            assert torch.equal(a["sd"][k], b["sd"][k]), k
    # blocking: nothing is ever outstanding at a compute instruction
    assert all(t[2] == 0 and t[3] == 0 for r in sync for t in r["trace"])
    # async: sends outstanding across compute on every stage that sends, and receives
    # posted ahead of a compute instruction on the stages that receive activations
    for rank, r in enumerate(asyn):
        if rank < stages - 1:
            assert any(t[2] > 0 for t in r["trace"]), (rank, r["trace"])
    assert any(t[3] > 0 for r in asyn[1:] for t in r["trace"] if t[0] == "BackwardPass")
