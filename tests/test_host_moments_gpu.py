"""Host-moments parameter groups (runtime/zero/sharded_base.py `_host_moments_step`): a param
group marked "host_moments" keeps its Adam moments in pinned host memory, streamed through HBM
per piece on copy engines beside the other groups' fused Adam.  Weights, losses and moments must
equal the all-HBM run bit for bit (same kernels on the same values), with the overlapped step and
without, compact fp32 master and plain fp32 master; checkpoints read the written-back moments."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29567")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _run(host, overlap, compact, steps=3, ga=2, piece=None):
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.runtime.zero import sharded_base
    if piece:
        sharded_base.ShardedOptimizerBase.HOST_PIECE = piece
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("gpt-neox-125m", num_layers=3, max_seq_len=128)
    model = GPTNeoX(cfg, device=dev, dtype=torch.bfloat16)
    tail = {id(p) for m in (model.embed_out, model.layers[-1]) for p in m.parameters()}
    groups = [{"params": [p for p in model.parameters() if id(p) not in tail]},
              {"params": [p for p in model.parameters() if id(p) in tail], "host_moments": host}]
    z = {"stage": 3, "reduce_bucket_size": int(5e6), "compact_master": compact, "overlap_step": overlap}
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": ga,
            "optimizer": {"type": "Adam", "params": {"lr": 3e-4}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "gradient_clipping": 1.0, "zero_optimization": z}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=groups, config_params=conf)
    opt = engine.optimizer
    on_host = [not opt.optimizer.state_for(g.master)["exp_avg"].is_cuda if hasattr(opt.optimizer, "state_for")
               else not opt.optimizer.state[g.master]["exp_avg"].is_cuda for g in opt.groups]
    g = torch.Generator(device=dev).manual_seed(7)
    losses = []
    for _ in range(steps):
        for _ in range(ga):
            ids = torch.randint(0, cfg.vocab_size, (2, 128), device=dev, generator=g)
            loss = engine(ids, labels=ids)
            engine.backward(loss)
            engine.step()
        losses.append(float(loss))
    engine.synchronize()
    sd = opt.state_dict()
    mom = [v["exp_avg_sq"].clone() for v in sd["base_optimizer_state"]["state"].values()]
    sharded_base.ShardedOptimizerBase.HOST_PIECE = int(16 * 1024 * 1024)
    return losses, [p.detach().float().cpu() for p in engine.module.parameters()], mom, on_host


@pytest.mark.parametrize("overlap,compact,mode,wgs", [(True, True, "stream", 0), (False, True, "stream", 0),
                                                      (True, False, "stream", 0), (True, True, "stream", 16),
                                                      (True, True, "side", 16), (True, True, "serial", 16)])
def test_host_moments_match_hbm_moments(overlap, compact, mode, wgs, monkeypatch):
    from deeperspeed_amd.runtime.zero import sharded_base
    monkeypatch.setattr(sharded_base, "HOST_STEP_MODE", mode)
    monkeypatch.setattr(sharded_base, "HOST_D2H_WGS", wgs)
    ref_l, ref_w, ref_m, ref_host = _run(False, overlap, compact)
    l, w, m, host = _run(True, overlap, compact, piece=300_000)  # several pieces per bucket: ring reuse
    assert ref_host == [False, False] and host == [False, True]
    assert l == ref_l
    for a, b in zip(ref_w, w):
        assert torch.equal(a, b)
    for a, b in zip(ref_m, m):
        assert torch.equal(a, b)


def test_copy_nocu_pinned_roundtrip():
    """DMA-engine copies (hipMemcpyDeviceToDeviceNoCU) between HBM and pinned host memory."""
    from deeperspeed_amd.ops import native
    x = torch.randn(3 * 1024 * 1024 + 7, device="cuda")
    h = torch.empty(x.numel(), dtype=torch.float32, pin_memory=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        native.copy_nocu_(h, x)
        y = torch.empty_like(x)
        native.copy_nocu_(y, h)
    s.synchronize()
    assert torch.equal(h, x.cpu())
    assert torch.equal(y, x)


@pytest.mark.parametrize("wgs", [1, 16, 64])
def test_copy_narrow_to_pinned(wgs):
    """copy_narrow_kernel: HBM -> pinned host on a few workgroups, odd byte tails included."""
    from deeperspeed_amd.ops import native
    for n in (1, 17, 4 * 1024 * 1024 + 3):
        x = torch.randint(0, 255, (n,), device="cuda", dtype=torch.uint8)
        h = torch.zeros(n, dtype=torch.uint8, pin_memory=True)
        native.copy_narrow_(h, x, wgs)
        torch.cuda.synchronize()
        assert torch.equal(h, x.cpu())
