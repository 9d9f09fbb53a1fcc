"""GPT-NeoX under ZeRO-3 with units small enough that attention / MLP sub-modules become
their own gather units (the 20B layout at unit_max_numel=2e8): 2 ranks on gloo must match
one rank.  Guards the rule that a module's weights are only used inside its own forward."""

import os

import pytest
import torch

from common import run_distributed


def _body(out_dir, world, unit, ckpt=False):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    torch.manual_seed(0)
    cfg = get_config("tiny", num_layers=2, checkpoint_activations=ckpt)
    model = GPTNeoX(cfg, dtype=torch.bfloat16)
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2 // world,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "fp32_allreduce": False, "zero_optimization": {"stage": 3, "stage3_unit_max_numel": unit,
                                                             "stage3_param_persistence_threshold": 0,
                                                             "reduce_bucket_size": 4096}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    g = torch.Generator().manual_seed(3)
    batches = [torch.randint(0, cfg.vocab_size, (2, 32), generator=g) for _ in range(2)]
    mine = batches[dist.get_rank()::world]
    losses = []
    for _ in range(3):
        tot = torch.zeros(())
        for ids in mine:
            loss = engine(ids, labels=ids)
            engine.backward(loss)
            engine.step()
            tot += loss.detach().float()
        dist.all_reduce(tot)
        losses.append(float(tot) / 2)
    if dist.get_rank() == 0:
        torch.save(losses, os.path.join(out_dir, f"w{world}_u{unit}_c{int(ckpt)}.pt"))


@pytest.mark.parametrize("unit,ckpt", [(20000, False), (70000, False), (20000, True)])
def test_neox_zero3_split_units(tmp_path, unit, ckpt):
    """ckpt=True: activation recompute with the output-projection skip, under ZeRO-3 hooks
    (the recomputed sub-module forwards re-gather; gradient-only projections still feed the
    reduce-scatter hooks)."""
    run_distributed(_body, 1, str(tmp_path), 1, unit, ckpt)
    run_distributed(_body, 2, str(tmp_path), 2, unit, ckpt)
    a = torch.load(tmp_path / f"w1_u{unit}_c{int(ckpt)}.pt")
    b = torch.load(tmp_path / f"w2_u{unit}_c{int(ckpt)}.pt")
    assert b[-1] < b[0]
    for x, y in zip(a, b):
        assert abs(x - y) < 2e-2 * max(1.0, abs(x)), (a, b)
