"""In-place weight-gradient accumulation (ops/linear.py): the wgrad GEMM accumulates into the
bound `p.grad` (beta = 1) and autograd still fires the post-accumulate hooks.  Checked
against stock autograd accumulation in fp32 at the layer level, and through the engine
(ZeRO-0/1/3, one and two gloo ranks, gradient accumulation) against DSA_FUSE_WGRAD off."""

import os

import pytest
import torch

from common import run_distributed


def test_linear_inplace_accumulate_matches_autograd():
    from deeperspeed_amd.ops import linear as lin
    torch.manual_seed(0)
    ref = torch.nn.Linear(16, 24)
    fused = lin.Linear(16, 24)
    fused.load_state_dict(ref.state_dict())
    fired = []
    fused.weight.register_post_accumulate_grad_hook(lambda p: fired.append("w"))
    fused.bias.register_post_accumulate_grad_hook(lambda p: fired.append("b"))
    # bind gradients as the engine does (flat arena views)
    arena = torch.zeros(24 * 16 + 24)
    fused.weight.grad = arena[: 24 * 16].view(24, 16)
    fused.bias.grad = arena[24 * 16:]
    xs = [torch.randn(3, 5, 16, requires_grad=True) for _ in range(3)]
    for x in xs:
        ref(x).square().sum().backward()
        x2 = x.detach().clone().requires_grad_(True)
        fused(x2).square().sum().backward()
        torch.testing.assert_close(x2.grad, x.grad)
    torch.testing.assert_close(fused.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(fused.bias.grad, ref.bias.grad, rtol=1e-5, atol=1e-5)
    assert fused.weight.grad.data_ptr() == arena.data_ptr()  # accumulated in place
    assert sorted(fired) == ["b"] * 3 + ["w"] * 3  # once per backward, by autograd


def test_linear_unbound_grad_falls_back():
    from deeperspeed_amd.ops import linear as lin
    torch.manual_seed(0)
    ref = torch.nn.Linear(8, 4, bias=False)
    fused = lin.Linear(8, 4, bias=False)
    fused.load_state_dict(ref.state_dict())
    x = torch.randn(6, 8)
    ref(x).sum().backward()
    fused(x).sum().backward()
    torch.testing.assert_close(fused.weight.grad, ref.weight.grad)


def _body(out_dir, world, stage, fuse):
    import torch.distributed as dist
    import deeperspeed_amd as ds
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.ops import linear as lin
    lin.FUSE_WGRAD = fuse
    n0 = lin.fused_wgrad_count()
    torch.manual_seed(0)
    cfg = get_config("tiny", num_layers=2)
    model = GPTNeoX(cfg, dtype=torch.bfloat16)
    zc = {"stage": stage, "reduce_bucket_size": 4096}
    if stage == 3:
        zc.update({"stage3_unit_max_numel": 20000, "stage3_param_persistence_threshold": 0})
    conf = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 4 // world,
            "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "fp16": {"enabled": True, "type": "bfloat16"},
            "zero_optimization": zc}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=conf)
    g = torch.Generator().manual_seed(3)
    batches = [torch.randint(0, cfg.vocab_size, (2, 32), generator=g) for _ in range(4)]
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
        losses.append(float(tot) / 4)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "fused_calls": lin.fused_wgrad_count() - n0},
                   os.path.join(out_dir, f"w{world}_s{stage}_f{int(fuse)}.pt"))


@pytest.mark.parametrize("stage,world", [(0, 1), (1, 2), (3, 1), (3, 2)])
def test_engine_fused_wgrad_equivalence(tmp_path, stage, world):
    run_distributed(_body, world, str(tmp_path), world, stage, False)
    run_distributed(_body, world, str(tmp_path), world, stage, True)
    a = torch.load(tmp_path / f"w{world}_s{stage}_f0.pt")
    b = torch.load(tmp_path / f"w{world}_s{stage}_f1.pt")
    assert a["fused_calls"] == 0
    assert b["fused_calls"] > 0, "fused wgrad path never ran"
    for x, y in zip(a["losses"], b["losses"]):
        assert abs(x - y) < 1e-2 * max(1.0, abs(x)), (a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("bound", [False, True])
def test_split_k_wgrad_matches_fp32(bound):
    """Small weights over many tokens take the split-K weight gradient (strided-batched partial
    GEMMs summed in fp32): fresh and bound (in-place accumulated) gradients match fp32."""
    from deeperspeed_amd.ops import linear as L
    torch.manual_seed(0)
    dev = torch.device("cuda")
    M, fin, fout = 8192, 1024, 1024
    assert L._split_k(torch.empty(M, fout, device=dev), torch.empty(M, fin, device=dev)) > 1
    x = torch.randn(M, fin, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = (0.02 * torch.randn(fout, fin, device=dev)).to(torch.bfloat16).requires_grad_(True)
    b = torch.zeros(fout, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g0 = torch.randn(fout, fin, device=dev, dtype=torch.bfloat16) if bound else None
    if bound:
        w.grad = g0.clone()
        b.grad = torch.zeros_like(b)
    dy = torch.randn(M, fout, device=dev, dtype=torch.bfloat16)
    L.linear(x, w, b).backward(dy)
    ref_w = dy.float().t() @ x.detach().float() + (g0.float() if bound else 0.0)
    ref_x = dy.float() @ w.detach().float()
    assert (w.grad.float() - ref_w).abs().max().item() < 2e-2 * ref_w.abs().max().item()
    assert (x.grad.float() - ref_x).abs().max().item() < 2e-2 * ref_x.abs().max().item()
    assert (b.grad.float() - dy.float().sum(0)).abs().max().item() < 2e-2 * dy.float().sum(0).abs().max().item()


@pytest.mark.gpu
def test_split_k_wgrad_as_accurate_as_one_gemm():
    """BERT-Large shape (8192 tokens, 1024x1024): the split-K weight gradient (fp32 partials,
    fp32 fold) is as close to the fp32 reference as a single GEMM with fp32 accumulation --
    both are one bf16 rounding of an fp32 sum."""
    from deeperspeed_amd.ops import linear as L
    torch.manual_seed(1)
    dev = torch.device("cuda")
    M, fin, fout = 8192, 1024, 1024
    x = torch.randn(M, fin, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, fout, device=dev, dtype=torch.bfloat16)
    s = L._split_k(dy, x)
    assert s > 1
    split = L._wgrad_split(dy, x, s)
    single = dy.t() @ x
    ref = dy.float().t() @ x.float()
    e_split = ((split.float() - ref).norm() / ref.norm()).item()
    e_single = ((single.float() - ref).norm() / ref.norm()).item()
    assert e_split <= 1.05 * e_single + 1e-6, (e_split, e_single)
    # the rounding floor of one bf16 cast of the exact result
    assert e_split < 3e-3, e_split
