"""Transposing bias+GeLU kernels (transpose.hip kGeluFwd / kGeluBwd) vs the row-major bias+GeLU
kernels and an fp32 PyTorch reference, and the GPT-NeoX MLP recompute that uses them (GeLU output
written column-major for fc2's weight gradient; du and du^T from one backward pass for fc1's)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("approx", [False, True])
@pytest.mark.parametrize("bias", [True, False])
def test_bias_gelu_fwd_t(dtype, approx, bias):
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    R, C = 384, 1216
    x = torch.randn(R, C, device=_dev(), dtype=dtype)
    b = torch.randn(C, device=_dev(), dtype=dtype) if bias else None
    yt = native.hip_ops().bias_gelu_fwd_t(x, b, approx)
    assert yt.shape == (C, R) and yt.is_contiguous()
    y = native.hip_ops().bias_gelu_fwd(x, b, approx)
    torch.testing.assert_close(yt.t(), y, atol=0, rtol=0)  # same math, same rounding
    ref = torch.nn.functional.gelu(x.float() + (b.float() if bias else 0), approximate="tanh" if approx else "none")
    torch.testing.assert_close(yt.t().float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("approx", [False, True])
@pytest.mark.parametrize("bias", [True, False])
def test_bias_gelu_bwd_t(dtype, approx, bias):
    from deeperspeed_amd.ops import native
    torch.manual_seed(1)
    R, C = 512, 768
    x = torch.randn(R, C, device=_dev(), dtype=dtype)
    dy = torch.randn(R, C, device=_dev(), dtype=dtype)
    b = torch.randn(C, device=_dev(), dtype=dtype) if bias else None
    dx, dxt, db = native.hip_ops().bias_gelu_bwd_t(dy, x, b, approx)
    dx0, db0 = native.hip_ops().bias_gelu_bwd(dy, x, b, approx)
    torch.testing.assert_close(dx, dx0, atol=0, rtol=0)
    torch.testing.assert_close(dxt, dx.t(), atol=0, rtol=0)
    xr = (x.float() + (b.float() if bias else 0)).requires_grad_(True)
    torch.nn.functional.gelu(xr, approximate="tanh" if approx else "none").backward(dy.float())
    torch.testing.assert_close(dx.float(), xr.grad, atol=3e-2, rtol=2e-2)
    if bias:
        torch.testing.assert_close(db.float(), xr.grad.sum(0), atol=0.25, rtol=2e-2)
    else:
        assert db is None or db.numel() == 0


def test_bias_gelu_colmajor_autograd():
    """Column-major GeLU output: same values as the row-major op, same gradients, and the
    backward offers du^T to the producing linear's weight gradient."""
    from deeperspeed_amd.ops import linear as lin
    from deeperspeed_amd.ops import native
    torch.manual_seed(2)
    x = torch.randn(2, 128, 1024, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(1024, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    y = native.bias_gelu_colmajor(x, b, False)
    assert y.shape == x.shape and not y.is_contiguous() and y.reshape(-1, 1024).t().is_contiguous()
    dy = torch.randn_like(y)
    y.backward(dy)
    x2 = x.detach().clone().requires_grad_(True)
    b2 = b.detach().clone().requires_grad_(True)
    y2 = native.bias_gelu(x2, b2, False)
    y2.backward(dy)
    torch.testing.assert_close(y, y2, atol=0, rtol=0)
    torch.testing.assert_close(x.grad, x2.grad, atol=0, rtol=0)
    torch.testing.assert_close(b.grad.float(), b2.grad.float(), atol=0.1, rtol=1e-2)
    lin.clear_transposed()


def _mlp_grads(colmajor, dual, monkeypatch, share=None):
    from deeperspeed_amd.models import gpt_neox
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.ops import linear as lin
    from deeperspeed_amd.ops import native
    monkeypatch.setattr(gpt_neox, "COLMAJOR_GELU", colmajor)
    monkeypatch.setattr(native, "DUAL_GELU_BWD", dual)
    monkeypatch.setattr(lin, "WGRAD_NT_MIN_NUMEL", 0)  # tiny weights take the transposed wgrad path
    monkeypatch.setattr(lin, "SHARE_GRAD_T", dual if share is None else share)
    torch.manual_seed(0)
    cfg = get_config("tiny", hidden_size=384, num_heads=4, num_layers=2, max_seq_len=128, checkpoint_activations=True)
    model = GPTNeoX(cfg, device="cuda", dtype=torch.bfloat16).train()
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
    nt0 = lin.nt_wgrad_count()
    loss = model(ids, labels=ids)
    loss.backward()
    assert lin.nt_wgrad_count() > nt0
    # every offered transpose (du^T for fc1; the block-output gradient^T that fc2 and the
    # attention output projection share) was consumed
    assert not lin._pre_t, [tuple(t.shape) for t, _ in lin._pre_t]
    return float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("share", [False, True])
def test_neox_recompute_colmajor_gelu_matches(monkeypatch, share):
    l0, g0 = _mlp_grads(False, False, monkeypatch)
    l1, g1 = _mlp_grads(True, True, monkeypatch, share)
    assert l0 == l1
    assert g0.keys() == g1.keys()
    for n in g0:
        scale = float(g0[n].abs().max()) + 1e-6
        torch.testing.assert_close(g1[n], g0[n], atol=2e-3 * scale, rtol=1e-2, msg=n)
