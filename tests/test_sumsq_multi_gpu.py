"""Multi-tensor sum of squares (ops/csrc/kernels/optim.hip sumsq_multi_kernel) against an fp64
torch reference: mixed sizes, odd lengths, misaligned views, every 16/32-bit dtype; and the global
gradient norm that the sync-free LAMB / unfused optimizer step is clipped with."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_sumsq_multi_matches_fp64(dtype):
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    base = torch.randn(300_001, device="cuda").to(dtype)
    ts = [torch.randn(n, device="cuda").to(dtype) for n in (1, 7, 64, 65_536, 65_537, 1_000_003)]
    ts += [base[3:70_003], base[1:2]]  # views not 16-byte aligned
    out = torch.zeros(1, device="cuda")
    native.sumsq_multi_(ts, out)
    ref = sum(float(t.double().square().sum()) for t in ts)
    assert abs(float(out) - ref) <= 1e-5 * ref
    native.sumsq_multi_(ts, out)  # accumulates (cached meta table)
    assert abs(float(out) - 2 * ref) <= 2e-5 * ref


def test_grad_norm_uses_hip_reduction():
    from deeperspeed_amd.runtime.utils import grad_norm_sq_tensor
    torch.manual_seed(1)
    ps = [torch.nn.Parameter(torch.randn(n, device="cuda", dtype=torch.bfloat16)) for n in (1024, 3, 70_000)]
    for p in ps:
        p.grad = torch.randn_like(p)
    sq = grad_norm_sq_tensor(ps)
    ref = sum(float(p.grad.double().square().sum()) for p in ps)
    assert abs(float(sq) - ref) <= 1e-5 * ref
