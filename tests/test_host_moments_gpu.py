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


@pytest.mark.parametrize("overlap,compact", [(True, True), (False, True), (True, False)])
def test_host_moments_match_hbm_moments(overlap, compact):
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


def _run_tiers(tiers, tmpdir, steps=3, ga=2):
    """offload_optimizer states='moments' with one param group per entry of `tiers`
    ("gpu" / "cpu" / "nvme" moments); None = no offload (all moments in HBM)."""
    _env()
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.runtime.zero import sharded_base
    sharded_base.ShardedOptimizerBase.NVME_PIECE = 200_000  # several pieces per bucket
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config("gpt-neox-125m", num_layers=3, max_seq_len=128)
    model = GPTNeoX(cfg, device=dev, dtype=torch.bfloat16)
    mods = [[model.embed_in, model.layers[0]], [model.layers[1]], [model.layers[2], model.final_layer_norm,
                                                                   model.embed_out]]
    groups = []
    for i, ms in enumerate(mods):
        pg = {"params": [p for m in ms for p in m.parameters()]}
        if tiers is not None:
            pg["moments_device"] = tiers[i]
        groups.append(pg)
    z = {"stage": 3, "reduce_bucket_size": int(5e6), "compact_master": True}
    if tiers is not None:
        z["offload_optimizer"] = {"device": "cpu", "pin_memory": True, "states": "moments",
                                  "nvme_path": str(tmpdir)}
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": ga,
            "optimizer": {"type": "Adam", "params": {"lr": 3e-4}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "gradient_clipping": 1.0, "zero_optimization": z}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=groups, config_params=conf)
    g = torch.Generator(device=dev).manual_seed(7)
    losses = []
    for _ in range(steps):
        for _ in range(ga):
            ids = torch.randint(0, cfg.vocab_size, (2, 128), device=dev, generator=g)
            loss = engine(ids, labels=ids)
            engine.backward(loss)
            engine.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    sd = engine.optimizer.state_dict()
    mom = [v["exp_avg_sq"].clone() for v in sd["base_optimizer_state"]["state"].values()]
    sharded_base.ShardedOptimizerBase.NVME_PIECE = int(32 * 1024 * 1024)
    return losses, [p.detach().float().cpu() for p in engine.module.parameters()], mom, engine


def test_three_tier_moments_match_hbm(tmp_path):
    """HBM / pinned-host / NVMe moment tiers (peak-params layout) equal the all-HBM step bit for
    bit, and a checkpoint written from the tiered optimizer restores into it exactly."""
    ref_l, ref_w, ref_m, _ = _run_tiers(None, tmp_path / "a")
    l, w, m, eng = _run_tiers(["gpu", "nvme", "cpu"], tmp_path / "b")
    assert eng.optimizer._mswap is not None and eng.optimizer._mswap.bytes_read > 0
    assert l == ref_l
    for a, b in zip(ref_w, w):
        assert torch.equal(a, b)
    for a, b in zip(ref_m, m):
        assert torch.equal(a, b)
    # round trip of the NVMe tier through state_dict / load_state_dict
    sd = eng.optimizer.state_dict()
    for gi in sd["base_optimizer_state"]["state"]:
        sd["base_optimizer_state"]["state"][gi]["exp_avg"] = sd["base_optimizer_state"]["state"][gi]["exp_avg"] + 1
    eng.optimizer.load_state_dict(sd)
    sd2 = eng.optimizer.state_dict()
    for gi in sd["base_optimizer_state"]["state"]:
        assert torch.equal(sd2["base_optimizer_state"]["state"][gi]["exp_avg"],
                           sd["base_optimizer_state"]["state"][gi]["exp_avg"])
