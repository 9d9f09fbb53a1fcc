"""Activation recompute skips the residual-branch output projections (their values are never
read by backward): gradients must match the non-checkpointed model exactly in fp32, for the
parallel-residual GPT-NeoX block, the sequential-residual variant (where the attention
projection must NOT be skipped) and GPT-2."""

import pytest
import torch


def _grads(model, ids):
    model.zero_grad(set_to_none=True)
    loss = model(ids, labels=ids)
    loss.backward()
    return float(loss.detach()), {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


def _compare(build, ids):
    torch.manual_seed(0)
    ref = build(False)
    torch.manual_seed(0)
    ck = build(True)
    ck.load_state_dict(ref.state_dict())
    l0, g0 = _grads(ref.train(), ids)
    l1, g1 = _grads(ck.train(), ids)
    assert abs(l0 - l1) < 1e-6
    assert g0.keys() == g1.keys()
    for k in g0:
        torch.testing.assert_close(g1[k], g0[k], rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("parallel", [True, False])
def test_neox_recompute_skip(parallel):
    from deeperspeed_amd.models import gpt_neox as gn
    from deeperspeed_amd.ops import linear as lin
    cfg_kw = dict(num_layers=2, max_seq_len=32, use_parallel_residual=parallel)
    ids = torch.randint(0, 512, (2, 32), generator=torch.Generator().manual_seed(1))
    calls = []
    orig = lin._GradOnlyLinear.forward

    def spy(ctx, x, w, b, *rest):
        calls.append(tuple(w.shape))
        return orig(ctx, x, w, b, *rest)

    lin._GradOnlyLinear.forward = staticmethod(spy)
    try:
        _compare(lambda ck: gn.GPTNeoX(gn.get_config("tiny", checkpoint_activations=ck, **cfg_kw)), ids)
    finally:
        lin._GradOnlyLinear.forward = staticmethod(orig)
    # 2 layers x (mlp out [+ attention out when the residual is parallel])
    assert len(calls) == (4 if parallel else 2)


def test_gpt2_recompute_skip():
    from deeperspeed_amd.models.gpt2 import GPT2, get_gpt2_config
    ids = torch.randint(0, 512, (2, 32), generator=torch.Generator().manual_seed(2))
    _compare(lambda ck: GPT2(get_gpt2_config("gpt2-tiny", checkpoint_activations=ck)), ids)
