"""Once-per-step weight transposes (ops/linear.py WeightTCache, opt-in): training through the engine with
the cache gives bit-identical weights to just-in-time transposes, the backward takes its W^T from
the cache, and an optimizer step (or an in-place weight write) invalidates it."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _train(cache_on, monkeypatch, steps=3):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.ops import linear as L
    monkeypatch.setattr(L, "WT_CACHE", cache_on)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("bert-large", num_layers=2, vocab_size=4096, max_position=128, hidden_dropout=0.0,
                     attn_dropout=0.0)
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": 8, "optimizer": {"type": "Lamb", "params": {"lr": 2e-3}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": 1.0}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    assert L.weight_t_cache.enabled == cache_on
    g = torch.Generator(device=dev).manual_seed(1)
    B, S, npred = 8, 128, 20
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    pos = torch.stack([torch.randperm(S, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)
    hits0, made0 = L.weight_t_cache.hits, L.weight_t_cache.made
    for _ in range(steps):
        loss = engine(ids, None, None, pos, lab, nsp)
        engine.backward(loss)
        engine.step()
    torch.cuda.synchronize()
    stats = (L.weight_t_cache.hits - hits0, L.weight_t_cache.made - made0)
    L.weight_t_cache.enable(False)
    return [p.detach().clone() for p in engine.module.parameters()], stats


def test_weight_t_cache_bit_identical(monkeypatch):
    w_off, st_off = _train(False, monkeypatch)
    w_on, st_on = _train(True, monkeypatch)
    assert st_off == (0, 0)
    # 4 linears per layer x 2 layers (+ the MLM dense / pooler are below the size floor):
    # one transpose made and one consumed per weight and step
    assert st_on[0] >= 8 * 3 and st_on[1] == st_on[0], st_on
    for a, b in zip(w_off, w_on):
        assert torch.equal(a, b)


def test_weight_t_cache_invalidation():
    from deeperspeed_amd.ops import linear as L
    from deeperspeed_amd.ops import native
    c = L.WeightTCache()
    c.enabled = True
    w = torch.randn(1024, 2048, device="cuda", dtype=torch.bfloat16)
    c.prepare(w, 4096)
    assert torch.equal(c.get(w), w.t())
    with torch.no_grad():
        w.mul_(2)  # in-place write: version counter moves
    assert c.get(w) is None
    c.prepare(w, 4096)
    assert torch.equal(c.get(w), w.t())
    native.hip_ops()  # raw-pointer writes (fused optimizers) are covered by the step epoch
    c.bump()
    assert c.get(w) is None
    c.prepare(w, 512)  # too few tokens for the transposed input gradient: not cached
    assert c.get(w) is None
