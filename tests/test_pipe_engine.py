"""Pipeline engine on gloo (reference analogue: tests/unit/test_pipe.py, test_pipe_module.py):
PP=2 and PP=2 x DP=2 must train to the same weights as a single-stage run of the same layers,
tied layers must stay tied, per-layer checkpoints must round-trip, and eval/inference
batches must return the DeeperSpeed outputs."""

import os

import pytest
import torch
import torch.nn as nn

from common import run_distributed

HID = 16


class _Act(nn.Module):
    def forward(self, x):
        return torch.relu(x)


def _lm_head(module, x):
    """GPT-NeoX-style tied output projection: the embedding module's weight, used differently."""
    return torch.nn.functional.linear(x, module.weight)


def _specs(tied=False):
    from deeperspeed_amd.runtime.pipe.module import LayerSpec, TiedLayerSpec
    specs = []
    if tied:
        specs.append(TiedLayerSpec("emb", nn.Linear, HID, HID))
    else:
        specs.append(LayerSpec(nn.Linear, HID, HID))
    for _ in range(4):
        specs += [LayerSpec(nn.Linear, HID, HID), LayerSpec(_Act)]
    if tied == "fn":
        specs.append(TiedLayerSpec("emb", nn.Linear, HID, HID, forward_fn=_lm_head))
    elif tied:
        specs.append(TiedLayerSpec("emb", nn.Linear, HID, HID))
    else:
        specs.append(LayerSpec(nn.Linear, HID, HID))
    return specs


def _data(n, seed):
    g = torch.Generator()
    g.manual_seed(seed)
    return [(torch.randn(4, HID, generator=g), torch.randint(0, HID, (4,), generator=g)) for _ in range(n)]


def _pipe_body(out_dir, num_stages, zero_stage, tied, steps=3, ga=4):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.pipe.module import PipelineModule
    torch.manual_seed(0)
    world = dist.get_world_size()
    dp = world // num_stages
    ga = 8 // dp  # global batch = 8 micro-batches for every topology
    model = PipelineModule(layers=_specs(tied), num_stages=num_stages, loss_fn=nn.CrossEntropyLoss(),
                           partition_method="uniform", seed_layers=True, base_seed=7)
    cfg = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": ga,
           "optimizer": {"type": "Adam", "params": {"lr": 1e-2}}, "steps_per_print": 1000,
           "fp16": {"enabled": True, "type": "bfloat16"}, "fp32_allreduce": False}
    if zero_stage:
        cfg["zero_optimization"] = {"stage": zero_stage}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=[p for p in model.parameters()],
                                    config_params=cfg)
    dp_rank = engine.grid.get_data_parallel_id()
    # one fixed global batch of 8 micro-batches, revisited every step (the model overfits it);
    # each data-parallel replica takes alternating micro-batches, a single replica takes all
    data = _data(8, 123)
    mine = data[dp_rank::2] if dp == 2 else data[0::2] + data[1::2]
    assert len(mine) == ga
    it = iter([(x.to(torch.bfloat16), y) for x, y in mine] * steps)
    losses = [float(engine.train_batch(it)) for _ in range(steps)]
    # gather the full model state on every rank for comparison
    sd = {}
    for idx, layer in enumerate(engine.module.forward_funcs):
        if hasattr(layer, "state_dict"):
            for k, v in layer.state_dict().items():
                sd[f"{idx + engine.module._local_start}.{k}"] = v.detach().float().clone()
    gathered = [None] * world
    dist.all_gather_object(gathered, sd)
    if dist.get_rank() == 0:
        full = {}
        for d in gathered:
            full.update(d)
        torch.save({"sd": full, "losses": losses}, os.path.join(out_dir, f"pp{num_stages}_z{zero_stage}_t{tied}.pt"))
    # per-layer checkpoint roundtrip
    engine.save_checkpoint(out_dir, tag="pipe")
    if dist.get_rank() == 0:
        files = os.listdir(os.path.join(out_dir, "pipe"))
        assert any(f.startswith("layer_00") for f in files) and "mp_rank_00_model_states.pt" in files
        last = len(_specs(tied)) - 1
        # a tied position with a forward_fn owns no layer file (reference pipe/module.py:546-567)
        assert any(f.startswith(f"layer_{last:02d}") for f in files) == (tied != "fn"), files
    engine2_model = PipelineModule(layers=_specs(tied), num_stages=num_stages, loss_fn=nn.CrossEntropyLoss(),
                                   partition_method="uniform", seed_layers=True, base_seed=99)
    e2, _, _, _ = ds.initialize(model=engine2_model, model_parameters=list(engine2_model.parameters()),
                                config_params=cfg)
    e2.load_checkpoint(out_dir, tag="pipe")
    for a, b in zip(engine.module.parameters(), e2.module.parameters()):
        assert torch.equal(a.detach(), b.detach())
    ev = e2.eval_batch(iter([(x.to(torch.bfloat16), y) for x, y in mine[:ga]]))
    assert torch.isfinite(ev)


@pytest.mark.parametrize("world,stages,zero", [(2, 2, 0), (4, 2, 1), (2, 1, 0)])
def test_pipeline_matches_reference(tmp_path, world, stages, zero):
    run_distributed(_pipe_body, world, str(tmp_path), stages, zero, False)
    res = torch.load(os.path.join(tmp_path, f"pp{stages}_z{zero}_tFalse.pt"), weights_only=True)
    assert res["losses"][-1] < res["losses"][0]


def test_pipeline_equivalence(tmp_path):
    os.makedirs(tmp_path / "a")
    os.makedirs(tmp_path / "b")
    run_distributed(_pipe_body, 2, str(tmp_path / "a"), 2, 0, False)
    run_distributed(_pipe_body, 1, str(tmp_path / "b"), 1, 0, False, 3, 8)
    a = torch.load(tmp_path / "a" / "pp2_z0_tFalse.pt", weights_only=True)
    b = torch.load(tmp_path / "b" / "pp1_z0_tFalse.pt", weights_only=True)
    for k in b["sd"]:
        assert torch.allclose(a["sd"][k], b["sd"][k], atol=3e-2, rtol=3e-2), k


@pytest.mark.parametrize("tied", [True, "fn"])
def test_pipeline_tied_layers(tmp_path, tied):
    run_distributed(_pipe_body, 2, str(tmp_path), 2, 0, tied)
    res = torch.load(os.path.join(tmp_path, f"pp2_z0_t{tied}.pt"), weights_only=True)
    assert res["losses"][-1] < res["losses"][0]


def _infer_body():
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.pipe.module import LayerSpec, PipelineModule

    class Head(nn.Module):
        def __init__(self):
            super().__init__()
            self.l = nn.Linear(HID, HID)

        def forward(self, x):
            logits = self.l(x)
            presents = torch.stack([logits, logits])
            return logits, presents

    specs = [LayerSpec(nn.Linear, HID, HID), LayerSpec(nn.Linear, HID, HID), LayerSpec(Head)]
    torch.manual_seed(0)
    model = PipelineModule(layers=specs, num_stages=2, loss_fn=None, partition_method="uniform")
    cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 1,
           "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=list(model.parameters()), config_params=cfg)
    x = torch.randn(2, HID)
    logits, presents = engine.inference_batch(iter([(x, torch.zeros(2))]))
    assert logits.shape == (2, HID) and presents.shape == (2, 2, HID)


def test_inference_batch_returns_logits_and_presents():
    run_distributed(_infer_body, 2)


def _module_plan(out):
    import torch.nn as nn
    from deeperspeed_amd.runtime.pipe.module import LayerSpec, PipelineModule, _plan_stages

    class Block(nn.Module):
        def __init__(self, d):
            super().__init__()
            self.lin = nn.Linear(d, d)

        def forward(self, x):
            return self.lin(x)

    specs = [LayerSpec(nn.Linear, 8, 64), LayerSpec(Block, 64), LayerSpec(Block, 64), LayerSpec(Block, 64),
             LayerSpec(Block, 64), LayerSpec(nn.Linear, 64, 8)]
    # type: balances the matching layers only; parameters balances trainable numel
    assert _plan_stages(specs, 2, "type:block") == [0, 3, 6]
    assert _plan_stages(specs, 2, "uniform") == [0, 3, 6]
    p = _plan_stages(specs, 3, "parameters")
    assert p[0] == 0 and p[-1] == 6 and len(p) == 4
    m = PipelineModule(layers=specs, num_stages=1, partition_method="type:Block", activation_checkpoint_interval=2,
                       checkpointable_layers=["Block"])
    # segments of 2: [Linear, Block] not checkpointable, [Block, Block] yes, [Block, Linear] no
    assert [(s.start, s.stop, s.recompute) for s in m._segments] == [(0, 2, False), (2, 4, True), (4, 6, False)]
    x = torch.randn(3, 8, requires_grad=True)
    y = m(x)
    y.sum().backward()
    assert y.shape == (3, 8) and x.grad is not None
    m.set_checkpoint_interval(0)
    assert [(s.start, s.stop, s.recompute) for s in m._segments] == [(0, 6, False)]


def test_pipeline_module_partition_and_segments():
    run_distributed(_module_plan, 1, None)
