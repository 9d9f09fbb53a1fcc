"""HBM rates of plain device copies, zero fills, reductions and the 2-D transpose kernel (calibration for the memory-bound HIP kernels)."""
import json, torch
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeperspeed_amd.ops import native
def t(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
x = torch.randn(8192, 18432, device="cuda", dtype=torch.bfloat16)
y = torch.empty_like(x)
nb = x.numel() * 2 * 2
ms = t(lambda: y.copy_(x)); print(json.dumps({"op": "copy_ 302MB", "ms": round(ms, 4), "TBps": round(nb / ms / 1e9, 2)}))
w = torch.randn(8192, 24576, device="cuda", dtype=torch.bfloat16)
nb2 = w.numel() * 4
ms = t(lambda: native.transpose2d(w)); print(json.dumps({"op": "transpose2d 8192x24576", "ms": round(ms, 4), "TBps": round(nb2 / ms / 1e9, 2)}))
ms = t(lambda: w.t().contiguous()); print(json.dumps({"op": "torch t().contiguous()", "ms": round(ms, 4), "TBps": round(nb2 / ms / 1e9, 2)}))
z = torch.empty(8192 * 18432 * 2, device="cuda", dtype=torch.bfloat16)
ms = t(lambda: z.zero_()); print(json.dumps({"op": "zero_ 604MB", "ms": round(ms, 4), "TBps": round(z.numel() * 2 / ms / 1e9, 2)}))
ms = t(lambda: x.sum()); print(json.dumps({"op": "sum read 302MB", "ms": round(ms, 4), "TBps": round(x.numel() * 2 / ms / 1e9, 2)}))

# compact-master Adam over one 77M-parameter group (the 20B step's per-group call): bytes moved per
# element: bf16 hi + int16 residual + bf16 grad + fp32 m, v read; hi, residual, m, v written
n = 77_000_000
hi = torch.randn(n, device="cuda").to(torch.bfloat16)
res = torch.zeros(n, device="cuda", dtype=torch.int16)
g = torch.randn(n, device="cuda").to(torch.bfloat16)
m = torch.zeros(n, device="cuda")
v = torch.zeros(n, device="cuda")
ops = native.hip_ops()
ms = t(lambda: ops.adam_compact(hi, res, g, m, v, 1e-4, 0.9, 0.95, 1e-8, 0.01, 0.1, 0.05, 1.0, True))
print(json.dumps({"op": "adam_compact 77M", "ms": round(ms, 4), "TBps": round(26 * n / ms / 1e9, 2)}))
