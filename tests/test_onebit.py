"""1-bit Adam / 1-bit LAMB and the compressed all-reduce on gloo (reference
tests/onebit/test_com_reduce_host.py, test_nccl_backend.py, tests/unit/test_onebit.py)."""

import os

import pytest
import torch

from common import run_distributed


def test_packbits_roundtrip_msb_first():
    from deeperspeed_amd.ops import native
    bits = torch.tensor([1, 0, 0, 0, 0, 0, 0, 1, 0, 1, 1, 1, 1, 1, 1, 1], dtype=torch.bool)
    packed = native._packbits(bits)
    assert packed.tolist() == [0b10000001, 0b01111111]
    assert torch.equal(native._unpackbits(packed) > 0, bits)


def _compressed_body(out_dir):
    import torch.distributed as dist
    from deeperspeed_amd.runtime.comm.nccl import NcclBackend
    rank, world = dist.get_rank(), dist.get_world_size()
    backend = NcclBackend()
    n = 8 * world * 50
    torch.manual_seed(rank)
    x = torch.randn(n)
    werr = torch.zeros(n)
    serr = torch.zeros(n // world)
    xs = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(xs, x)
    exact = torch.stack(xs).mean(0)
    out = backend.compressed_allreduce(x.clone(), werr, serr, rank)
    # every rank gets the same result, and the worker error closes the loop:
    # out == mean over ranks of (x_r - err_r) up to the server compression error
    outs = [torch.empty_like(out) for _ in range(world)]
    dist.all_gather(outs, out)
    for o in outs:
        assert torch.equal(o, outs[0])
    # error feedback: repeated compression of the same tensor converges to the exact mean
    acc = torch.zeros(n)
    for _ in range(30):
        acc += backend.compressed_allreduce(x.clone(), werr, serr, rank)
    err = (acc / 30 - exact).abs().mean() / exact.abs().mean()
    if rank == 0:
        torch.save(float(err), os.path.join(out_dir, "err.pt"))


def test_compressed_allreduce_error_feedback(tmp_path):
    run_distributed(_compressed_body, 2, str(tmp_path))
    assert torch.load(tmp_path / "err.pt") < 0.15


def _onebit_body(out_dir, opt_type):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from simple_model import SimpleModel, random_batches
    torch.manual_seed(0)
    model = SimpleModel(16)
    params = {"lr": 1e-2, "freeze_step": 3}
    cfg = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 1,
           "optimizer": {"type": opt_type, "params": params}, "fp16": {"enabled": True, "type": "bfloat16"}}
    engine, opt, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    data = random_batches(1, 4, 16, seed=1 + dist.get_rank()) * 10
    losses = []
    for i, (x, y) in enumerate(data):
        loss = engine(x.to(torch.bfloat16), y)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.detach()))
        if i >= 3:
            assert engine.enable_backward_allreduce is False  # compression stage
    flat = torch.cat([p.detach().float().view(-1) for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.allclose(flat, other, atol=1e-2), "replicas diverged"
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("opt_type", ["OneBitAdam", "OneBitLamb"])
def test_onebit_optimizer_trains(opt_type):
    run_distributed(_onebit_body, 2, None, opt_type)
