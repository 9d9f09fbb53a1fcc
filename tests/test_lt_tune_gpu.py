"""GPU numerics of the measured-solution GEMM routes (ops/lt_tune.py, ops/csrc/gemm_lt.cpp).

Each route is checked against a plain fp32 PyTorch reference of the same op at a GPT-NeoX-20B
shape that the shipped table covers (8192 tokens, 6144 x 6144 attention output projection).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

M, N, K = 8192, 6144, 6144


def _ops():
    from deeperspeed_amd.ops import linear
    return linear._lt_ops()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.fixture(scope="module")
def data():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    return x, w, b, dy


def test_table_covers_the_tested_shape():
    from deeperspeed_amd.ops import lt_tune
    t = lt_tune.load_table()
    for kind, bias in (("fwd", True), ("dgrad", False), ("wgrad", False)):
        assert lt_tune.key(kind, M, N, K, bias) in t, kind


def test_forward_with_bias(data):
    x, w, b, _ = data
    y = _ops().linear_lt(x, w, b, None, False, None)
    ref = x.float() @ w.float().t() + b.float()
    assert _rel(y, ref) < 1e-2


def test_input_gradient_nn(data):
    _, w, _, dy = data
    dx = _ops().gemm_lt(dy, w)
    ref = dy.float() @ w.float()
    assert _rel(dx, ref) < 1e-2


def test_weight_gradient_nt_accumulates(data):
    x, _, _, dy = data
    g0 = (torch.randn(N, K, device=x.device) * 10).to(torch.bfloat16)
    g = g0.clone()
    _ops().gemm_lt(dy, x, trans_a=True, out=g, accumulate=True)
    ref = g0.float() + dy.float().t() @ x.float()
    assert _rel(g, ref) < 1e-2


def test_choices_recorded_and_table_candidates_timed(data):
    choices = _ops().lt_choices()
    assert choices, "no tuned problem recorded"
    # every tuned problem of this module had the table's solutions among its candidates
    # (heuristic 16 at most + registered ones)
    for c in choices:
        ta, tb, m, n, k, epi, has_c, idx, ms, cand, registered, name = c
        assert cand >= 1 and name


def test_linear_layer_routes_match_reference(data, monkeypatch):
    """ops.linear forward + backward (bound weight / bias gradients) through the forward route."""
    from deeperspeed_amd.ops import linear, lt_tune
    monkeypatch.setattr(lt_tune, "ENABLED", True)
    monkeypatch.setattr(lt_tune, "FWD", True)
    x0, w0, b0, dy = data
    x = x0.clone().requires_grad_(True)
    w = torch.nn.Parameter(w0.clone())
    b = torch.nn.Parameter(b0.clone())
    w.grad = torch.zeros_like(w)
    b.grad = torch.zeros_like(b)
    y = linear.linear(x, w, b)
    y.backward(dy)
    xf, wf = x0.float(), w0.float()
    assert _rel(y, xf @ wf.t() + b0.float()) < 1e-2
    assert _rel(x.grad, dy.float() @ wf) < 1e-2
    assert _rel(w.grad, dy.float().t() @ xf) < 1e-2
    assert _rel(b.grad, dy.float().sum(0)) < 1e-2
