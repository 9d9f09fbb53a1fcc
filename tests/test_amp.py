"""`amp` config block -> torch autocast with fp32 masters, loss scaling, clipping and the initial
model broadcast (REF deepspeed/runtime/engine.py:643,682-693,1085-1093,1146-1155); legacy
`deepspeed.pt.*` import paths (REF deepspeed/__init__.py:39-49)."""

import importlib

import pytest
import torch
import torch.nn as nn

import deeperspeed_amd as ds
from tests.common import distributed_test


class _Net(nn.Module):
    def __init__(self, d=16):
        super().__init__()
        self.a = nn.Linear(d, d)
        self.b = nn.Linear(d, 4)
        self.seen = []

    def forward(self, x, y):
        h = self.a(x)
        self.seen.append(h.dtype)
        return nn.functional.cross_entropy(self.b(torch.relu(h)).float(), y)


def _conf(**amp):
    return {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 1,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-2, "torch_adam": True}},
            "gradient_clipping": 1.0, "amp": dict(enabled=True, **amp)}


def _engine(conf, seed=0):
    torch.manual_seed(seed)
    net = _Net()
    eng, _, _, _ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=conf)
    return eng, net


def test_amp_runs_forward_under_autocast_with_fp32_masters():
    eng, net = _engine(_conf())
    x, y = torch.randn(4, 16), torch.randint(0, 4, (4,))
    loss = eng(x, y)
    assert net.seen[-1] == torch.bfloat16  # matmul ran in bf16
    assert all(p.dtype == torch.float32 for p in net.parameters())  # masters stay fp32
    w0 = net.a.weight.detach().clone()
    eng.backward(loss)
    eng.step()
    assert not torch.equal(w0, net.a.weight)
    assert eng.amp is not None and eng.amp.scaler is None


def test_amp_clips_gradients(monkeypatch):
    eng, net = _engine(_conf())
    seen = {}
    from deeperspeed_amd.runtime import engine as engine_mod
    real = engine_mod.clip_grad_norm_

    def spy(parameters, max_norm, **kw):
        seen["max_norm"] = max_norm
        return real(parameters=parameters, max_norm=max_norm, **kw)

    monkeypatch.setattr(engine_mod, "clip_grad_norm_", spy)
    x, y = torch.randn(4, 16) * 100, torch.randint(0, 4, (4,))
    eng.backward(eng(x, y))
    eng.step()
    assert seen.get("max_norm") == 1.0


def test_amp_fp16_dynamic_scaler_skips_overflow():
    eng, net = _engine(_conf(dtype="float16", init_scale=2.0 ** 10))
    assert eng.amp.scaler is not None
    x, y = torch.randn(4, 16), torch.randint(0, 4, (4,))
    loss = eng(x, y)
    eng.backward(loss)
    # poison one gradient: the step must be skipped and counted, the scale backed off
    net.a.weight.grad[0, 0] = float("inf")
    w0 = net.a.weight.detach().clone()
    eng.step()
    assert torch.equal(w0, net.a.weight)
    assert eng.skipped_steps == 1
    assert eng.amp.loss_scale < 2.0 ** 10


def test_amp_fp16_static_scale_counts_overflow():
    """a fixed loss_scale builds (no GradScaler factor assert), keeps its scale, and a
    non-finite gradient still skips and counts the step."""
    eng, net = _engine(_conf(dtype="float16", loss_scale=128))
    assert eng.amp.loss_scale == 128.0
    x, y = torch.randn(4, 16), torch.randint(0, 4, (4,))
    eng.backward(eng(x, y))
    w0 = net.a.weight.detach().clone()
    eng.step()
    assert not torch.equal(w0, net.a.weight) and eng.skipped_steps == 0
    eng.backward(eng(x, y))
    net.a.weight.grad[0, 0] = float("nan")
    w1 = net.a.weight.detach().clone()
    eng.step()
    assert torch.equal(w1, net.a.weight)
    assert eng.skipped_steps == 1
    assert eng.amp.loss_scale == 128.0


def test_amp_o0_is_plain_fp32():
    eng, net = _engine(_conf(opt_level="O0"))
    eng(torch.randn(4, 16), torch.randint(0, 4, (4,)))
    assert net.seen[-1] == torch.float32


def test_amp_rejects_zero():
    conf = _conf()
    conf["zero_optimization"] = {"stage": 1}
    with pytest.raises(AssertionError, match="ZeRO"):
        _engine(conf)


def test_amp_state_checkpoint_roundtrip(tmp_path):
    eng, _ = _engine(_conf(dtype="float16", init_scale=512.0))
    eng.backward(eng(torch.randn(4, 16), torch.randint(0, 4, (4,))))
    eng.step()
    eng.save_checkpoint(str(tmp_path), tag="t")
    eng2, _ = _engine(_conf(dtype="float16", init_scale=4.0), seed=1)
    eng2.load_checkpoint(str(tmp_path), tag="t")
    assert eng2.amp.loss_scale == eng.amp.loss_scale


@distributed_test(world_size=2)
def _amp_broadcast_body():
    import torch.distributed as dist
    eng, net = _engine(_conf(), seed=100 + dist.get_rank())  # different init on every rank
    w = net.a.weight.detach().clone()
    ws = [torch.empty_like(w) for _ in range(2)]
    dist.all_gather(ws, w)
    assert torch.equal(ws[0], ws[1]), "amp must not skip the initial model broadcast"


def test_amp_broadcasts_model_world2(monkeypatch):
    monkeypatch.delenv("DSA_SKIP_MODEL_BROADCAST", raising=False)
    _amp_broadcast_body()


@pytest.mark.parametrize("name,target", [("deepspeed_utils", "deeperspeed_amd.runtime.utils"),
                                         ("deepspeed_config", "deeperspeed_amd.runtime.config"),
                                         ("loss_scaler", "deeperspeed_amd.runtime.fp16.loss_scaler")])
def test_legacy_pt_aliases(name, target):
    mod = importlib.import_module("deepspeed.pt." + name)
    assert mod is importlib.import_module(target)
    import deepspeed
    assert getattr(deepspeed.pt, name) is mod
