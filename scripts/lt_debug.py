"""Print how the hipBLASLt wrapper tunes one GPT-NeoX-20B linear (run with DSA_LT_DEBUG=1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from deeperspeed_amd.ops import linear  # noqa: E402

M, N, K = 8192, 6144, 6144
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.01
b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
ops = linear._lt_ops()
ops.linear_lt(x, w, b, None, False, None)
ops.gemm_lt(dy, w)
g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
ops.gemm_lt(dy, x, trans_a=True, out=g, accumulate=True)
torch.cuda.synchronize()
for c in ops.lt_choices():
    print(c)
