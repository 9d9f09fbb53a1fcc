"""Layer-batched weight gradients (ops/wgrad_batch.py): the slab / gradient-stack bookkeeping and
the batched flush against per-record GEMMs, a weight used twice in one backward, and BERT training
through the engine with and without batching."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_flush_batches_consecutive_slots():
    from deeperspeed_amd.ops import wgrad_batch as wb
    g = torch.Generator().manual_seed(0)
    L, M, N, K = 4, 1024, 384, 256
    wb.state.slabs.clear()
    wb.state.stacks.clear()
    wb.enable(True)
    try:
        xs = [wb.view("x", i, L, torch.empty(M, K, device="cuda", dtype=torch.bfloat16)) for i in range(L)]
        dys = [wb.view("dy", i, L, torch.empty(M, N, device="cuda", dtype=torch.bfloat16), backward=True)
               for i in range(L)]
        assert all(t is not None for t in xs + dys)
        assert wb.view("dy", 0, L, dys[0], backward=True) is None  # lent until release()
        for t in xs + dys:
            t.copy_(torch.randn(t.shape, generator=g).to(t.dtype))
        ps = [torch.nn.Parameter(torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)) for _ in range(L)]
        assert wb.bind_grad_stacks(ps, min_numel=1) == L
        for p in ps:
            p.grad.copy_(torch.randn(N, K, generator=g).to(torch.bfloat16))
        ref = [p.grad.float() + d.float().t() @ x.float() for p, d, x in zip(ps, dys, xs)]
        b0 = wb.state.batched
        with wb.deferred(True):
            for i in (2, 0, 3, 1):  # recorded out of order
                wb.record(dys[i], xs[i], ps[i].grad)
        assert wb.state.batched == b0 + 1 and not wb.state.pending
        for p, r in zip(ps, ref):
            assert (p.grad.float() - r).abs().max().item() <= 1e-2 * r.abs().max().item()
        assert wb.view("dy", 0, L, dys[0], backward=True) is not None  # released at the end of the pass
    finally:
        wb.enable(False)
        wb.release()


def test_deferred_weight_used_twice():
    from deeperspeed_amd.ops import linear as L
    from deeperspeed_amd.ops import wgrad_batch as wb
    torch.manual_seed(0)
    lin = L.Linear(256, 256).cuda().bfloat16()
    other = L.Linear(256, 256).cuda().bfloat16()
    x0 = torch.randn(2048, 256, device="cuda", dtype=torch.bfloat16)
    grads = {}
    wb.enable(True)
    try:
        for defer in (False, True):
            for p in list(lin.parameters()) + list(other.parameters()):
                p.grad = torch.zeros_like(p)  # bound gradients, as the engine binds them
            slot = wb.view("twice", 0, 2, x0)  # the input in a slab slot: its gradients may be deferred
            slot.copy_(x0)
            x = slot.detach().requires_grad_(True)
            r0 = wb.state.recorded
            with wb.deferred(defer):
                y = lin(other(lin(x)))  # lin's weight gradient is recorded for its first use
                y.float().pow(2).mean().backward()
            wb.release()
            assert (wb.state.recorded > r0) == defer and not wb.state.pending
            grads[defer] = [p.grad.float().clone() for p in list(lin.parameters()) + list(other.parameters())]
    finally:
        wb.enable(False)
    for a, b in zip(grads[False], grads[True]):
        assert (a - b).abs().max().item() <= 2e-2 * max(1e-3, a.abs().max().item())


def _env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29573")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _train(batch, monkeypatch, steps=3):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.ops import wgrad_batch as wb
    monkeypatch.setattr(wb, "ENABLED", batch)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("bert-large", num_layers=4, vocab_size=4096, max_position=128)  # dropout 0.1
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": 8, "optimizer": {"type": "Lamb", "params": {"lr": 2e-3}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": 1.0}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    assert engine._defer_wgrad == batch
    g = torch.Generator(device=dev).manual_seed(1)
    B, S, npred = 8, 128, 20
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    am = torch.ones(B, S, device=dev, dtype=torch.long)
    am[:, 100:] = 0
    pos = torch.stack([torch.randperm(100, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)
    b0, losses = wb.state.batched, []
    for _ in range(steps):
        loss = engine(ids, None, am, pos, lab, nsp)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.detach()))
    torch.cuda.synchronize()
    out = losses, [p.detach().float().clone() for p in engine.module.parameters()], wb.state.batched - b0
    print("last batching miss:", wb.state.last_miss, "slabs:", {k: v.key[:2] for k, v in wb.state.slabs.items()},
          "recorded:", wb.state.recorded, "single:", wb.state.single)
    wb.enable(False)
    return out


def test_bert_training_with_batched_wgrads(monkeypatch):
    l0, w0, n0 = _train(False, monkeypatch)
    l1, w1, n1 = _train(True, monkeypatch)
    # qkv / attn-out / fc1 / fc2 every step
    assert n0 == 0 and n1 >= 4 * 3, (n0, n1)
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 2e-2 * abs(a)
    for a, b in zip(w0, w1):
        assert (a - b).abs().max().item() <= 1e-2 * max(1.0, a.abs().max().item())


def test_graph_captured_params_are_not_rebound():
    """Parameters whose addresses a HIP graph holds (make_graphed_encoder) keep their .grad and
    storage: rebinding them to stacks would leave the graph writing into freed memory."""
    from deeperspeed_amd.ops import wgrad_batch as wb
    ps = [torch.nn.Parameter(torch.zeros(256, device="cuda", dtype=torch.bfloat16)) for _ in range(4)]
    grads = [torch.ones_like(p) for p in ps]
    for p, g in zip(ps, grads):
        p.grad = g
        p._dsa_graph_captured = True
    n0 = len(wb.state.stacks)
    assert wb.bind_grad_stacks(ps, min_numel=1) == 0 and len(wb.state.stacks) == n0
    assert all(p.grad is g for p, g in zip(ps, grads))
    free = [torch.nn.Parameter(torch.zeros(256, device="cuda", dtype=torch.bfloat16)) for _ in range(4)]
    free[0].grad = torch.full_like(free[0], 3.0)
    try:
        assert wb.bind_grad_stacks(free, min_numel=1) == 4
        assert torch.all(free[0].grad == 3.0) and free[1].grad.data_ptr() - free[0].grad.data_ptr() == 512
    finally:
        del wb.state.stacks[n0:]


def _bert_engine(batch, monkeypatch, dropout=0.0, pld=False):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.ops import wgrad_batch as wb
    monkeypatch.setattr(wb, "ENABLED", batch)
    wb.state.slabs.clear()
    wb.state.off_kinds.clear()
    wb.state.reshapes.clear()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("bert-large", num_layers=4, vocab_size=4096, max_position=256, hidden_dropout=dropout,
                     attn_dropout=dropout)
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": 8, "optimizer": {"type": "Lamb", "params": {"lr": 2e-3}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": 1.0}
    if pld:
        conf["progressive_layer_drop"] = {"enabled": True, "theta": 0.5, "gamma": 0.01}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    assert engine._defer_wgrad == batch
    return engine, cfg, dev


def _bert_batch(cfg, dev, seed, B=8, S=128):
    g = torch.Generator(device=dev).manual_seed(seed)
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    am = torch.ones(B, S, device=dev, dtype=torch.long)
    pos = torch.stack([torch.randperm(S - 8, device=dev, generator=g)[:20].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, 20), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)
    return ids, None, am, pos, lab, nsp


def test_interleaved_forwards_keep_their_slots(monkeypatch):
    """fwd A (takes the slots), fwd B (ordinary memory), bwd B, fwd C, bwd A.  The end of
    bwd B must not free A's slots, or fwd C overwrites the activations bwd A reads (silently: the
    kernels write slots through raw out= pointers).  Gradients must equal the unbatched engine's."""
    from deeperspeed_amd.ops import wgrad_batch as wb
    grads = {}
    for batch in (False, True):
        engine, cfg, dev = _bert_engine(batch, monkeypatch)
        a, b, c = (_bert_batch(cfg, dev, s) for s in (1, 2, 3))
        la = engine(*a)
        lb = engine(*b)
        engine.backward(lb)
        lc = engine(*c)  # noqa: F841 - its graph is never backpropagated
        engine.backward(la)
        torch.cuda.synchronize()
        grads[batch] = [p.grad.float().clone() for p in engine.module.parameters() if p.grad is not None]
        if batch:
            assert wb.state.recorded > 0
        wb.enable(False)
    assert len(grads[False]) == len(grads[True])
    for x, y in zip(grads[False], grads[True]):
        assert (x - y).abs().max().item() <= 2e-2 * max(1e-3, x.abs().max().item())


def test_slab_memory_flat_under_pld_and_shape_changes(monkeypatch):
    """slabs are keyed per kind -- progressive layer drop (a different kept-layer count
    every step) and a seq-128 / seq-256 switch must not allocate a fresh set of slabs per shape."""
    from deeperspeed_amd.ops import wgrad_batch as wb
    engine, cfg, dev = _bert_engine(True, monkeypatch, pld=True)
    peaks = []
    for step in range(10):
        S = 128 if step % 2 == 0 else 256
        loss = engine(*_bert_batch(cfg, dev, step, S=S))
        engine.backward(loss)
        engine.step()
        torch.cuda.synchronize()
        peaks.append(torch.cuda.memory_allocated())
    kinds = len(wb.state.slabs)
    wb.enable(False)
    # after the first few steps the unstable kinds are off and nothing more is allocated
    assert max(peaks[4:]) <= peaks[3] + (64 << 20), [p >> 20 for p in peaks]
    assert kinds <= 16
