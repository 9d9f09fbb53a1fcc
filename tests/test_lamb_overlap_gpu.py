"""Overlapped LAMB step (zero_optimization.overlap_step on the per-tensor FP16_UnfusedOptimizer
path, runtime/overlap_step.py): the fused LAMB of step k runs on a side stream in forward-ordered
buckets while the forward of step k+1 starts; every module waits only for its own bucket.  The
result must equal the serial step bit for bit -- including the BERT MLM decoder that reads the
tied word-embedding weight outside the embedding module (covered by the calibration pass)."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29563")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _train(overlap, clip, steps=4, bucket_numel=None, graphs=False):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.runtime.fp16.unfused_optimizer import FP16_UnfusedOptimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("bert-large", num_layers=3, vocab_size=4096, max_position=128, hidden_dropout=0.0,
                     attn_dropout=0.0)
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    conf = {"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 1,
            "optimizer": {"type": "Lamb", "params": {"lr": 2e-3, "weight_decay": 0.01}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": clip,
            "zero_optimization": {"stage": 0, "overlap_step": overlap}}
    if graphs:  # graphed before initialize: overlap_step's forward pre-hooks come after the capture
        from deeperspeed_amd.ops.transformer.transformer import make_graphed_encoder
        B, S = 8, 128
        ext = torch.zeros(B, 1, 1, S, device=dev, dtype=torch.bfloat16)
        make_graphed_encoder(model.layers, torch.randn(B, S, cfg.hidden_size, device=dev, dtype=torch.bfloat16), ext)
        for p in model.parameters():  # the capture's warmup iterations accumulated into them
            if p.grad is not None:
                p.grad.zero_()
        torch.cuda.synchronize()
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    opt = engine.optimizer
    assert isinstance(opt, FP16_UnfusedOptimizer)
    assert (opt._overlap is not None) == overlap
    g = torch.Generator(device=dev).manual_seed(1)
    B, S, npred = 8, 128, 20
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
    tt = (torch.arange(S, device=dev)[None] >= S // 2).long().expand(B, S).contiguous()
    am = torch.ones(B, S, device=dev, dtype=torch.long)
    pos = torch.stack([torch.randperm(S, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
    lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
    nsp = torch.randint(0, 2, (B,), device=dev, generator=g)
    losses = []
    for _ in range(steps):
        loss = engine(ids, tt, am, pos, lab, nsp)
        engine.backward(loss)
        engine.step()
        losses.append(loss.detach())
    engine.synchronize()
    norms = opt.get_global_grad_norm()
    w = [p.detach().float().cpu() for p in engine.module.parameters()]
    st = [opt.state[m]["exp_avg_sq"].cpu() for g_ in opt.fp32_groups for m in g_]
    return [float(x) for x in losses], w, st, norms, len(getattr(opt, "_overlap_buckets", []))


@pytest.mark.parametrize("clip", [0.0, 0.05])
def test_overlapped_lamb_step_is_exact(clip):
    base_l, base_w, base_s, _, _ = _train(False, clip)
    ov_l, ov_w, ov_s, _, nb = _train(True, clip)
    assert nb > 3  # forward-ordered buckets, not one
    assert base_l == ov_l
    for a, b in zip(base_w, ov_w):
        assert torch.equal(a, b)
    for a, b in zip(base_s, ov_s):
        assert torch.equal(a, b)
    assert base_l[-1] < base_l[0]


def test_overlapped_lamb_with_hip_graph_persistent_grads():
    """HIP-graphed encoder (persistent .grad buffers zeroed in place) + overlapped step: the side
    stream zeroes each bucket's persistent buffers behind its own LAMB kernels, so the next
    replay never accumulates into a buffer the step is still reading.  Must equal
    graphed + serial step bit for bit."""
    base_l, base_w, base_s, _, _ = _train(False, 1.0, steps=5, graphs=True)
    ov_l, ov_w, ov_s, _, _ = _train(True, 1.0, steps=5, graphs=True)
    assert base_l == ov_l
    for a, b in zip(base_w, ov_w):
        assert torch.equal(a, b)
    for a, b in zip(base_s, ov_s):
        assert torch.equal(a, b)


def test_lamb_device_scale_skips_non_finite():
    """The device-resident gradient factor of the overlapped step: a NaN factor leaves weights
    and moments untouched; a finite one equals the host-scalar grad_scale."""
    from deeperspeed_amd.ops.lamb.fused_lamb import FusedLamb
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ws = [torch.randn(n, device=dev) for n in (1000, 70000, 8)]
    gs = [torch.randn(w.shape, device=dev, dtype=torch.bfloat16) for w in ws]

    def run(scale_t, host_scale):
        ps = [torch.nn.Parameter(w.clone()) for w in ws]
        opt = FusedLamb(ps, lr=1e-2, weight_decay=0.01)
        if scale_t is None:
            opt.step(grads=[gs], scale=1.0 / host_scale)
        else:
            opt.step_subset(0, list(range(len(ps))), gs, None, scale_t)
        torch.cuda.synchronize()
        return [p.detach().clone() for p in ps], [opt.state[p]["exp_avg"].clone() for p in ps]

    w_host, m_host = run(None, 0.37)
    w_dev, m_dev = run(torch.tensor([0.37], device=dev), None)
    for a, b in zip(w_host + m_host, w_dev + m_dev):
        assert torch.equal(a, b)
    w_nan, m_nan = run(torch.tensor([float("nan")], device=dev), None)
    for a, w in zip(w_nan, ws):
        assert torch.equal(a, w)
    for m in m_nan:
        assert torch.count_nonzero(m).item() == 0


@pytest.mark.parametrize("clip", [0.0, 0.05])
def test_sync_free_step_matches_host_checked_step(monkeypatch, clip):
    """bf16 LAMB step with the clip factor formed on the device (no host read of the norm) vs the
    host-checked step: identical without clipping, equal to fp32 rounding of the factor with."""
    from deeperspeed_amd.runtime.fp16 import unfused_optimizer as uo
    monkeypatch.setattr(uo, "SYNC_FREE_STEP", False)
    host_l, host_w, _, host_n, _ = _train(False, clip, steps=3)
    monkeypatch.setattr(uo, "SYNC_FREE_STEP", True)
    dev_l, dev_w, _, dev_n, _ = _train(False, clip, steps=3)
    assert abs(host_n - dev_n) <= 1e-3 * host_n
    if clip == 0.0:
        assert host_l == dev_l
        for a, b in zip(host_w, dev_w):
            assert torch.equal(a, b)
    else:
        for a, b in zip(host_l, dev_l):
            assert abs(a - b) <= 1e-3 * abs(a)
        for a, b in zip(host_w, dev_w):
            assert torch.allclose(a, b, rtol=1e-2, atol=1e-3)


def test_sync_free_skip_is_counted_and_rolled_back():
    """a sync-free bf16 LAMB step with a non-finite gradient is skipped inside the
    kernels; the engine learns it at the next print / checkpoint boundary (skipped_steps), and the
    per-parameter step counters are rolled back so later bias corrections are right."""
    _env()
    import torch.nn as nn
    import deeperspeed_amd as ds
    from deeperspeed_amd.runtime.fp16 import unfused_optimizer as uo
    if not uo.SYNC_FREE_STEP:
        pytest.skip("DSA_SYNC_FREE_STEP=0")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(256, 512), nn.GELU(), nn.Linear(512, 256)).to(dev, torch.bfloat16)
    conf = {"train_micro_batch_size_per_gpu": 8, "gradient_accumulation_steps": 1, "steps_per_print": 3,
            "optimizer": {"type": "Lamb", "params": {"lr": 1e-3}},
            "fp16": {"enabled": True, "type": "bfloat16"}, "gradient_clipping": 1.0}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    opt = engine.optimizer
    assert isinstance(opt, uo.FP16_UnfusedOptimizer) and opt._sync_free([p for g in opt.fp16_groups for p in g])
    x = torch.randn(8, 256, device=dev, dtype=torch.bfloat16)
    for i in range(3):
        loss = engine(x).float().pow(2).mean()
        engine.backward(loss)
        if i == 1:
            next(iter(model.parameters())).grad[0, 0] = float("inf")
        engine.step()
    torch.cuda.synchronize()
    assert engine.skipped_steps == 1  # reconciled at the steps_per_print boundary
    steps = {st["step"] for st in opt.state.values() if "step" in st}
    assert steps == {2}
