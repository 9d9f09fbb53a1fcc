"""ZeRO communication modes (gloo/CPU, the same code that runs on RCCL):

* ZeRO-3 `stage3_force_sharded` on a world of one runs the gather / reduce-scatter path and
  must reproduce the bind-to-shard bypass bit for bit;
* `resident_grads` (ZeRO-2 / 3) cuts the gradient reductions to one per optimizer step
  (a factor of gradient_accumulation_steps) without changing the result;
* `reduce_scatter: false` (all-reduce, reference parity), `overlap_comm: false` and
  `sub_group_size` stepping give the same weights as the defaults;
* stage 0 (the flat-arena mixed-precision wrapper) is pinned to `torch.optim.AdamW` on an
  unsharded fp32 master.

Reference analogue: tests/unit/test_zero.py / test_fp16.py stage matrices.
"""

import os

import torch

from common import run_distributed
from simple_model import LinearStack, SimpleModel, base_config, random_batches


def _count_collectives():
    """Wrap the framework's collective entry points with per-op counters."""
    from deeperspeed_amd.utils import comm
    counts = {"reduce_scatter": 0, "all_reduce": 0, "all_gather": 0}
    for name, key in (("reduce_scatter_tensor", "reduce_scatter"), ("all_reduce", "all_reduce"),
                      ("all_gather_into_tensor", "all_gather")):
        orig = getattr(comm, name)

        def wrapped(*a, _orig=orig, _key=key, **kw):
            if "norm" not in kw.get("tag", ""):
                counts[_key] += 1
            return _orig(*a, **kw)
        setattr(comm, name, wrapped)
    return counts


def _train(out_dir, tag, stage, ga, zero, steps=3, hidden=32, model="stack", fp32_reduce=False, dtype="bfloat16",
           lr=1e-2, eps=None):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    counts = _count_collectives()
    torch.manual_seed(7)
    net = LinearStack(input_dim=hidden, hidden_dim=48, output_dim=hidden, num_layers=3) if model == "stack" \
        else SimpleModel(hidden)
    cfg = base_config(stage=stage, mb=4, ga=ga, dtype=dtype, lr=lr, **zero)
    if eps is not None:
        cfg["optimizer"]["params"]["eps"] = eps
    xdt = torch.bfloat16 if dtype == "bfloat16" else torch.float32
    if fp32_reduce:
        cfg["fp32_allreduce"] = True
    if stage == 0:
        cfg.pop("zero_optimization", None)
    engine, _, _, _ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=cfg)
    rank = dist.get_rank()
    data = random_batches(steps * ga, 4, hidden, seed=100 + rank)
    losses = []
    for k, (x, y) in enumerate(data):
        loss = engine(x.to(xdt), y)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss.detach()))
    if stage == 3:
        sd = engine.optimizer.gathered_state_dict(engine.module)
    else:
        sd = {k: v.detach().cpu().clone() for k, v in engine.module.state_dict().items()}
    masters = [engine.optimizer.master_fp32(g).float() for g in engine.optimizer.groups]
    if rank == 0:
        torch.save({"sd": sd, "losses": losses, "counts": dict(counts), "masters": masters},
                   os.path.join(out_dir, f"{tag}.pt"))


def _load(tmp_path, tag):
    return torch.load(os.path.join(tmp_path, f"{tag}.pt"), weights_only=True)


def _same(a, b, exact):
    for k in a["sd"]:
        x, y = a["sd"][k].float(), b["sd"][k].float()
        if exact:
            assert torch.equal(x, y), k
        else:
            assert torch.allclose(x, y, atol=2e-2, rtol=2e-2), k


ZBASE = {"reduce_bucket_size": 700, "stage3_unit_max_numel": 2500, "stage3_param_persistence_threshold": 10,
         "reduce_scatter": True}


def test_zero3_force_sharded_matches_bypass(tmp_path):
    """World of one: the sharded unit machinery == the bind-to-shard bypass, bit for bit."""
    run_distributed(_train, 1, str(tmp_path), "bypass_ga1", 3, 1, dict(ZBASE))
    run_distributed(_train, 1, str(tmp_path), "sharded_ga1", 3, 1, dict(ZBASE, stage3_force_sharded=True))
    a, b = _load(tmp_path, "bypass_ga1"), _load(tmp_path, "sharded_ga1")
    assert a["losses"] == b["losses"]
    _same(a, b, exact=True)
    assert b["counts"]["all_gather"] > 0 and b["counts"]["reduce_scatter"] > 0
    assert a["counts"]["all_gather"] == 0 and a["counts"]["reduce_scatter"] == 0
    # gradient accumulation: resident unit grads accumulate in the parameter dtype exactly
    # like the bypass accumulates into the bound shard
    run_distributed(_train, 1, str(tmp_path), "bypass_ga2", 3, 2, dict(ZBASE))
    run_distributed(_train, 1, str(tmp_path), "sharded_ga2", 3, 2,
                    dict(ZBASE, stage3_force_sharded=True, resident_grads=True, grad_accum_dtype="param"))
    a, b = _load(tmp_path, "bypass_ga2"), _load(tmp_path, "sharded_ga2")
    assert a["losses"] == b["losses"]
    _same(a, b, exact=True)


def test_resident_grads_one_reduction_per_step(tmp_path):
    """GA x fewer gradient reductions with the same result: in fp32 (Adam eps 1e-3, see
    test_zero_fp32_exact.py) resident unit gradients summed before one reduction per step and
    per-micro-batch reductions agree to fp32 rounding."""
    ga, lr = 4, 1e-2
    for stage in (2, 3):
        run_distributed(_train, 2, str(tmp_path), f"s{stage}_plain", stage, ga, dict(ZBASE), lr=lr, dtype="float32",
                        eps=1e-3)
        run_distributed(_train, 2, str(tmp_path), f"s{stage}_res", stage, ga, dict(ZBASE, resident_grads=True),
                        lr=lr, dtype="float32", eps=1e-3)
        a, b = _load(tmp_path, f"s{stage}_plain"), _load(tmp_path, f"s{stage}_res")
        n_plain, n_res = a["counts"]["reduce_scatter"], b["counts"]["reduce_scatter"]
        assert n_plain > 0 and n_plain == ga * n_res, (stage, n_plain, n_res)
        for ma, mb in zip(a["masters"], b["masters"]):
            assert (ma - mb).abs().max() <= 1e-6, (stage, (ma - mb).abs().max())
        assert abs(a["losses"][-1] - b["losses"][-1]) < 1e-6


def test_reduce_scatter_false_and_overlap_off_match(tmp_path):
    for stage in (2, 3):
        run_distributed(_train, 2, str(tmp_path), f"s{stage}_rs", stage, 2, dict(ZBASE), dtype="float32", eps=1e-3)
        run_distributed(_train, 2, str(tmp_path), f"s{stage}_ar", stage, 2,
                        dict(ZBASE, reduce_scatter=False, overlap_comm=False), dtype="float32", eps=1e-3)
        a, b = _load(tmp_path, f"s{stage}_rs"), _load(tmp_path, f"s{stage}_ar")
        assert b["counts"]["reduce_scatter"] == 0 and b["counts"]["all_reduce"] > 0
        for k in a["sd"]:
            assert (a["sd"][k].float() - b["sd"][k].float()).abs().max() <= 1e-6, k


def test_sub_group_size_stepping_is_exact(tmp_path):
    run_distributed(_train, 2, str(tmp_path), "sg_big", 3, 1, dict(ZBASE))
    run_distributed(_train, 2, str(tmp_path), "sg_small", 3, 1, dict(ZBASE, sub_group_size=128))
    a, b = _load(tmp_path, "sg_big"), _load(tmp_path, "sg_small")
    _same(a, b, exact=True)


def _stage0_vs_adamw():
    """Stage 0 bf16 on 2 ranks vs torch.optim.AdamW on an fp32 master fed the fp32 average of
    both ranks' bf16 gradients (what fp32_allreduce computes)."""
    import torch.distributed as dist
    import deeperspeed_amd as ds
    hidden, steps, lr, wd = 16, 4, 1e-2, 0.1
    torch.manual_seed(3)
    net = SimpleModel(hidden)
    ref_master = [p.detach().to(torch.bfloat16).float() for p in net.parameters()]  # engine casts the module
    cfg = base_config(stage=0, mb=4, lr=lr)
    cfg["optimizer"]["params"].update(weight_decay=wd, betas=[0.9, 0.99], eps=1e-8)
    cfg["fp32_allreduce"] = True
    cfg.pop("zero_optimization", None)
    engine, _, _, _ = ds.initialize(model=net, model_parameters=net.parameters(), config_params=cfg)
    # reference: an unsharded fp32 master stepped by torch AdamW; forward/backward in bf16
    shadow = SimpleModel(hidden).to(torch.bfloat16)
    masters = [torch.nn.Parameter(m) for m in ref_master]
    opt = torch.optim.AdamW(masters, lr=lr, betas=(0.9, 0.99), eps=1e-8, weight_decay=wd)
    batches = [random_batches(steps, 4, hidden, seed=500 + r) for r in range(2)]
    rank = dist.get_rank()
    for s in range(steps):
        x, y = batches[rank][s]
        loss = engine(x.to(torch.bfloat16), y)
        engine.backward(loss)
        engine.step()
        grads = None
        for r in range(2):
            with torch.no_grad():
                for p, m in zip(shadow.parameters(), masters):
                    p.copy_(m.to(torch.bfloat16))
            shadow.zero_grad()
            xr, yr = batches[r][s]
            shadow(xr.to(torch.bfloat16), yr).backward()
            g = [p.grad.float() for p in shadow.parameters()]
            grads = g if grads is None else [a + b for a, b in zip(grads, g)]
        for m, g in zip(masters, grads):
            m.grad = g / 2
        opt.step()
    zo = engine.optimizer
    for p, m in zip(engine.module.parameters(), masters):
        g, b, i = zo._pos[p]
        lo = b.shard_offset + b.offsets[i]
        got = zo.master_fp32(g)[lo: lo + b.numels[i]]
        assert torch.allclose(got, m.detach().reshape(-1), atol=1e-5, rtol=1e-5), (got, m)


def test_stage0_matches_torch_adamw():
    run_distributed(_stage0_vs_adamw, 2)
