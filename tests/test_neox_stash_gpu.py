"""Selective recompute (NeoXAttention.stash_outputs): the first forward of a checkpointed block
keeps q, k, v and the flash output + LSE; the recompute reuses them.  Gradients must equal the
full-recompute ones (same kernels, same inputs: bitwise up to GEMM ordering)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(stash_layers, offload=False, sparse=None):
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    torch.manual_seed(0)
    extra = {"sparse_attention": {"mode": sparse, "block": 16}} if sparse else {}
    cfg = get_config("tiny", hidden_size=384, num_heads=4, num_layers=3, max_seq_len=128,
                     checkpoint_activations=True, **extra)
    model = GPTNeoX(cfg, device="cuda", dtype=torch.bfloat16).train()
    layers = [m for m in model.modules() if type(m).__name__ == "NeoXTransformerLayer"]
    for m in layers[:stash_layers]:
        m.attention.stash_outputs = True
        m.attention.stash_offload = offload
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
    for _ in range(2):  # second pass reuses nothing stale from the first
        model.zero_grad(set_to_none=True)
        loss = model(ids, labels=ids)
        loss.backward()
    assert all(not m.attention._stash for m in layers), "stash not consumed by the recompute"
    return float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("offload", [False, True])
def test_stash_matches_full_recompute(offload):
    """HBM stash, and the stash parked in pinned host memory (D2H on a copy stream, prefetched
    back by the recompute of the layer above) give the full-recompute gradients."""
    l0, g0 = _grads(0)
    l1, g1 = _grads(3 if offload else 2, offload)
    assert l0 == l1
    assert g0.keys() == g1.keys()
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n], atol=1e-3, rtol=1e-3, msg=n)


@pytest.mark.parametrize("sparse", ["bigbird", "fixed"])
def test_sparse_stash_matches_full_recompute(sparse):
    """Block-sparse attention (fused LUT kernels): the stashed (o, lse) of the first forward
    give the full-recompute gradients."""
    l0, g0 = _grads(0, sparse=sparse)
    l1, g1 = _grads(2, sparse=sparse)
    assert l0 == l1
    assert g0.keys() == g1.keys()
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n], atol=1e-3, rtol=1e-3, msg=n)


@pytest.mark.parametrize("offload", [False, True])
def test_stash_two_forwards_before_backward(offload):
    """Two checkpointed forwards in flight (pipeline 1F1B pattern): each backward must
    recompute with its own micro-batch's stash."""
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config

    def run(stash):
        torch.manual_seed(0)
        cfg = get_config("tiny", hidden_size=384, num_heads=4, num_layers=2, max_seq_len=128,
                         checkpoint_activations=True)
        model = GPTNeoX(cfg, device="cuda", dtype=torch.bfloat16).train()
        for m in model.modules():
            if type(m).__name__ == "NeoXAttention":
                m.stash_outputs = stash
                m.stash_offload = stash and offload
        g = torch.Generator(device="cuda").manual_seed(3)
        a = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
        b = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
        la, lb = model(a, labels=a), model(b, labels=b)
        la.backward()
        ga = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
        model.zero_grad(set_to_none=True)
        lb.backward()
        gb = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
        return ga, gb

    ra, rb = run(False)
    sa, sb = run(True)
    for n in ra:
        torch.testing.assert_close(sa[n], ra[n], atol=1e-3, rtol=1e-3, msg=n)
        torch.testing.assert_close(sb[n], rb[n], atol=1e-3, rtol=1e-3, msg=n)


def test_mlp_stash_matches_full_recompute():
    """MLP selective recompute (NeoXMLP.stash_outputs): the recompute takes the fc1 output the first
    forward kept (gradient-only fc1 GEMM) -- same gradients as the full recompute, also combined
    with the attention stash."""
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config

    def run(att, mlp):
        torch.manual_seed(0)
        cfg = get_config("tiny", hidden_size=384, num_heads=4, num_layers=3, max_seq_len=128,
                         checkpoint_activations=True)
        model = GPTNeoX(cfg, device="cuda", dtype=torch.bfloat16).train()
        for m in model.layers:
            m.attention.stash_outputs = att
            m.mlp.stash_outputs = mlp
        g = torch.Generator(device="cuda").manual_seed(1)
        ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
        for _ in range(2):
            model.zero_grad(set_to_none=True)
            loss = model(ids, labels=ids)
            loss.backward()
        assert all(not m.mlp._stash and not m.attention._stash for m in model.layers)
        return float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}

    l0, g0 = run(False, False)
    for att in (False, True):
        l1, g1 = run(att, True)
        assert l0 == l1
        for n in g0:
            torch.testing.assert_close(g1[n], g0[n], atol=1e-3, rtol=1e-3, msg=n)
