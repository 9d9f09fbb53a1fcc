"""FusedLamb (reference tests/unit/test_fp16.py lamb cases): CPU math vs a plain PyTorch LAMB
written from the paper/reference semantics, and engine training with fp16/bf16 + LAMB on 2
ranks (FP16_UnfusedOptimizer path)."""

import math

import pytest
import torch

from common import distributed_test, run_distributed

import deeperspeed_amd as ds


def _ref_lamb(w, g, m, v, lr, b1, b2, eps, wd, step, maxc, minc):
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    u = m / (v.sqrt() + eps) + wd * w
    wn, un = w.norm().item(), u.norm().item()
    c = 1.0 if (wn == 0 or un == 0) else min(max(wn / un, minc), maxc)
    ss = lr * math.sqrt(1 - b2 ** step) / (1 - b1 ** step)
    w.sub_(ss * c * u)
    return c


def test_fused_lamb_matches_reference_math():
    from deeperspeed_amd.ops.lamb import FusedLamb
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(300))
    q = p.detach().clone()
    m, v = torch.zeros(300), torch.zeros(300)
    opt = FusedLamb([p], lr=1e-2, weight_decay=0.01)
    for step in range(1, 6):
        g = torch.randn(300)
        p.grad = g.clone()
        opt.step()
        c = _ref_lamb(q, g, m, v, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, 10.0, 0.01)
        assert abs(opt.get_lamb_coeffs()[0] - c) < 1e-5
    assert torch.allclose(p.detach(), q, atol=1e-6)


def _engine_body(dtype):
    import deeperspeed_amd as ds
    from simple_model import SimpleModel, random_batches
    import torch.distributed as dist
    torch.manual_seed(0)
    model = SimpleModel(16)
    cfg = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 1,
           "optimizer": {"type": "Lamb", "params": {"lr": 1e-2}}, "gradient_clipping": 1.0,
           "fp16": {"enabled": True, "type": dtype, "loss_scale": 0 if dtype == "fp16" else 1.0}}
    engine, opt, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    assert type(opt).__name__ == "FP16_UnfusedOptimizer"
    losses = []
    for x, y in random_batches(1, 4, 16, seed=1) * 12:
        loss = engine(x.to(torch.bfloat16 if dtype == "bfloat16" else torch.float16), y)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0]
    # replicas stay identical
    flat = torch.cat([p.detach().float().view(-1) for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)


@pytest.mark.parametrize("dtype", ["bfloat16"])
def test_engine_lamb_unfused(dtype):
    run_distributed(_engine_body, 2, dtype)


@distributed_test(world_size=2)
def _reconcile_every_rank_body(tmpdir):
    """the sync-free LAMB step's device-side skip count is reconciled -- and the
    optimizer's step counters rolled back -- on EVERY rank at the print / checkpoint boundary, not
    only on the reporting rank, so replicated parameters keep identical bias corrections."""
    import torch.distributed as dist
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 2)).to(torch.bfloat16)
    conf = {"train_micro_batch_size_per_gpu": 2, "steps_per_print": 2,
            "optimizer": {"type": "Lamb", "params": {"lr": 1e-3}}, "fp16": {"enabled": True, "type": "bfloat16"}}
    eng, opt, _, _ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=conf)
    assert hasattr(opt, "reconcile_skipped_steps")
    x = torch.randn(2, 8, dtype=torch.bfloat16)
    for i in range(4):
        eng.backward(eng(x).float().pow(2).mean())
        if i == 0:  # the kernels skipped one step on the device (emulated: CPU has no sync-free path)
            opt._dev_skipped = torch.ones(1, dtype=torch.int32)
        eng.step()
    steps = [st["step"] for st in opt.state.values() if "step" in st]
    mine = torch.tensor([eng.skipped_steps, min(steps), max(steps)], dtype=torch.float64)
    both = [torch.empty_like(mine) for _ in range(2)]
    dist.all_gather(both, mine)
    assert torch.equal(both[0], both[1]), both
    assert int(mine[0]) == 1
    eng.save_checkpoint(tmpdir, tag="t")  # the checkpoint boundary reconciles on every rank as well


def test_reconcile_device_skips_on_every_rank(tmp_path):
    _reconcile_every_rank_body(str(tmp_path))
