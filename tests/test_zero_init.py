"""deeperspeed_amd.zero surface on gloo (reference tests/unit/test_zero_context.py,
test_zero_tiled.py, test_zero.py external-params cases)."""

import os

import pytest
import torch
import torch.nn as nn

from common import run_distributed
from simple_model import LinearStack, base_config, random_batches


def _cfg(stage=3, **z):
    zz = {"stage3_unit_max_numel": 3000, "stage3_param_persistence_threshold": 0, "reduce_bucket_size": 2048}
    zz.update(z)
    return base_config(stage=stage, mb=4, ga=1, **zz)


def _train(engine, steps=4, seed=0):
    import torch.distributed as dist
    data = random_batches(1, 4, 32, seed=seed + dist.get_rank(), classes=16) * steps
    out = []
    for x, y in data:
        loss = engine(x.to(torch.bfloat16), y)
        engine.backward(loss)
        engine.step()
        out.append(float(loss.detach()))
    return out


def _init_body(out_dir, use_init):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    torch.manual_seed(5)
    if use_init:
        with ds.zero.Init():
            model = LinearStack()
        p = model.input_layer.weight
        assert p.numel() == 0 and p.ds_numel == 64 * 32 and p.ds_tensor.numel() == (64 * 32 + 1) // 2
    else:
        model = LinearStack()
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=_cfg())
    losses = _train(engine)
    sd = engine.optimizer.gathered_state_dict(engine.module)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "sd": sd}, os.path.join(out_dir, f"init{int(use_init)}.pt"))


def test_zero_init_matches_eager(tmp_path):
    run_distributed(_init_body, 2, str(tmp_path), False)
    run_distributed(_init_body, 2, str(tmp_path), True)
    a = torch.load(tmp_path / "init0.pt", weights_only=True)
    b = torch.load(tmp_path / "init1.pt", weights_only=True)
    assert a["losses"] == pytest.approx(b["losses"], rel=1e-3)
    for k in a["sd"]:
        assert torch.allclose(a["sd"][k].float(), b["sd"][k].float(), atol=1e-3), k


def _gathered_body():
    import torch.distributed as dist
    import deeperspeed_amd as ds
    torch.manual_seed(0)
    model = LinearStack()
    engine, opt, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=_cfg())
    w = model.layers[1].weight
    assert w.numel() == 0  # released between uses
    with ds.zero.GatheredParameters(w, modifier_rank=0):
        assert w.shape == (64, 64)
        if dist.get_rank() == 0:
            w.data.fill_(0.5)
    assert w.numel() == 0
    sd = opt.gathered_state_dict(engine.module)
    assert torch.all(sd["layers.1.weight"] == 0.5)
    # the fp32 master follows the edit: one zero-lr step keeps the value
    masters = torch.cat([opt.master_fp32(g) for g in opt.groups])
    assert (masters == 0.5).sum() >= (64 * 64) // 2 - 64


def test_gathered_parameters_modifier_rank():
    run_distributed(_gathered_body, 2)


class _TiedHead(nn.Module):
    """Uses the embedding weight of another module in its forward (tied LM head)."""

    def __init__(self, emb):
        super().__init__()
        self.emb = [emb]  # not a registered submodule
        self.ln = nn.LayerNorm(32)

    def forward(self, x):
        return self.ln(x) @ self.emb[0].weight


class _TiedModel(nn.Module):
    def __init__(self):
        super().__init__()
        import deeperspeed_amd as ds
        self.embed = nn.Linear(16, 32, bias=False)
        self.body = nn.Linear(32, 32)
        self.head = _TiedHead(self.embed)
        self.loss = nn.MSELoss()
        ds.zero.register_external_parameter(self.head, self.embed.weight)

    def forward(self, x, y):
        h = torch.relu(self.body(self.embed(x)))
        out = self.head(h)  # [B, 16]
        return self.loss(out.float(), y.float())


def _external_body():
    import deeperspeed_amd as ds
    torch.manual_seed(0)
    model = _TiedModel()
    cfg = _cfg(stage3_unit_max_numel=600)
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    x = torch.randn(4, 16).to(torch.bfloat16)
    y = torch.randn(4, 16)
    losses = []
    for _ in range(5):
        loss = engine(x, y)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < losses[0]


def test_register_external_parameter():
    run_distributed(_external_body, 2)


def test_tiled_linear_matches_dense():
    from deeperspeed_amd.zero import TiledLinear, TiledLinearReturnBias
    torch.manual_seed(0)
    dense = nn.Linear(37, 23)
    t = TiledLinear(37, 23, in_splits=3, out_splits=2, init_linear=dense)
    x = torch.randn(5, 37)
    torch.testing.assert_close(t(x), dense(x), atol=1e-5, rtol=1e-5)
    tb = TiledLinearReturnBias(37, 23, in_splits=2, out_splits=3, init_linear=dense)
    y, b = tb(x)
    torch.testing.assert_close(y + b, dense(x), atol=1e-5, rtol=1e-5)
    parts = TiledLinear(37, 23, in_splits=2, out_splits=1, input_is_already_split=True, init_linear=dense)
    torch.testing.assert_close(parts(list(torch.split(x, parts.in_parts, -1))), dense(x), atol=1e-5, rtol=1e-5)


def test_linear_zero3_function_grads():
    from deeperspeed_amd.zero import LinearModuleForZeroStage3
    torch.manual_seed(0)
    a = nn.Linear(12, 7)
    b = LinearModuleForZeroStage3(12, 7)
    b.load_state_dict(a.state_dict())
    x = torch.randn(3, 4, 12, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    a(x).square().sum().backward()
    b(x2).square().sum().backward()
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(a.weight.grad, b.weight.grad)
    torch.testing.assert_close(a.bias.grad, b.bias.grad)


def test_contiguous_memory_allocator_defragments():
    from deeperspeed_amd.zero import ContiguousMemoryAllocator
    alloc = ContiguousMemoryAllocator(100, torch.float32, "cpu")
    ts = [alloc.allocate_tensor(20) for _ in range(5)]
    params = []
    for i, t in enumerate(ts):
        t.fill_(i)
        p = nn.Parameter(torch.empty(0))
        alloc.assign_to_param(t, p, 20, (4, 5))
        params.append(p)
    alloc.release_tensor(ts[1])
    alloc.release_tensor(ts[3])
    assert alloc.largest_contiguous == 20
    big = alloc.allocate_tensor(40)  # forces compaction
    big.fill_(9)
    for i in (0, 2, 4):
        assert torch.all(params[i] == i) and params[i].shape == (4, 5)
    assert alloc.total_free == 0 and alloc.max_allocated() == 100
