"""hipBLASLt epilogue GEMMs (ops/csrc/gemm_lt.cpp) against fp32 PyTorch references."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_linear_lt_bias_residual_gelu(dtype):
    from deeperspeed_amd.ops import native
    ops = native.hip_ops()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    M, K, N = 512, 256, 384
    x = torch.randn(M, K, device=dev, dtype=dtype)
    w = torch.randn(N, K, device=dev, dtype=dtype) * 0.05
    b = torch.randn(N, device=dev, dtype=dtype)
    r = torch.randn(M, N, device=dev, dtype=dtype)
    ref = x.float() @ w.float().t() + b.float()
    y = ops.linear_lt(x, w, b, None, False, None)
    assert (y.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    y = ops.linear_lt(x, w, b, r, False, None)
    assert (y.float() - (ref + r.float())).abs().max().item() < 3e-2 * ref.abs().max().item()
    y = ops.linear_lt(x, w, b, None, True, None)
    g = F.gelu(ref, approximate="tanh")
    assert (y.float() - g).abs().max().item() < 3e-2 * g.abs().max().item()


def test_epilogue_probe_reports_available_forms():
    from deeperspeed_amd.ops import native
    ops = native.hip_ops()
    assert ops.lt_algo_count(1024, 512, 256, 4, False) > 0    # BIAS
    assert ops.lt_algo_count(1024, 512, 256, 36, False) > 0   # GELU_BIAS


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_lt_layouts_and_accumulate(ta, tb):
    """General autotuned GEMM: every operand layout, fresh output and in-place accumulate."""
    from deeperspeed_amd.ops import native
    ops = native.hip_ops()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    M, K, N = 384, 256, 320
    a = torch.randn(K, M, device=dev, dtype=torch.bfloat16) if ta else torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=dev, dtype=torch.bfloat16) if tb else torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    c = ops.gemm_lt(a, b, ta, tb)
    assert c.shape == (M, N)
    assert (c.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    acc = torch.randn(M, N, device=dev, dtype=torch.float32)
    want = acc + ref
    ops.gemm_lt(a, b, ta, tb, acc, True)
    assert (acc - want).abs().max().item() < 1e-3 * want.abs().max().item()
