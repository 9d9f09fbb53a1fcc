"""bias + GeLU forward / backward HIP kernels at the BERT-Large (8192 x 4096) and GPT-NeoX-20B
(8192 x 24576) fc1 shapes: time per call, effective HBM rate, and the error against torch's fp32
GeLU of the same inputs.

    python scripts/bench_gelu.py [--approx 1] [--shapes 8192x4096,8192x24576]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from deeperspeed_amd.ops import native  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--approx", type=int, default=1)
    ap.add_argument("--shapes", default="8192x4096,8192x24576")
    args = ap.parse_args()
    ops = native.hip_ops()
    approx = bool(args.approx)
    for shp in args.shapes.split(","):
        R, C = (int(v) for v in shp.split("x"))
        g = torch.Generator(device="cuda").manual_seed(0)
        x = (torch.randn(R, C, device="cuda", generator=g) * 2).bfloat16()
        b = (torch.randn(C, device="cuda", generator=g) * 0.1).bfloat16()
        dy = torch.randn(R, C, device="cuda", generator=g).bfloat16()
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        db = torch.zeros(C, device="cuda", dtype=torch.bfloat16)
        t_f = timed(lambda: ops.bias_gelu_fwd(x, b, approx, y))
        t_b = timed(lambda: ops.bias_gelu_bwd(dy, x, b, approx, dx, None))
        t_ft = timed(lambda: ops.bias_gelu_fwd_t(x, b, approx))  # transposed output (recompute path)
        t_bt = timed(lambda: ops.bias_gelu_bwd_t(dy, x, b, approx))  # du and du^T + bias sums
        xf = (x.float() + b.float()).requires_grad_(True)
        ref = F.gelu(xf, approximate="tanh" if approx else "none")
        ref.backward(dy.float())
        ops.bias_gelu_fwd(x, b, approx, y)
        ops.bias_gelu_bwd(dy, x, b, approx, dx, None)
        ef = ((y.float() - ref.detach()).abs().max() / ref.detach().abs().max()).item()
        eb = ((dx.float() - xf.grad).abs().max() / xf.grad.abs().max()).item()
        n = R * C * 2
        print(json.dumps({"R": R, "C": C, "approx": approx, "fwd_us": round(t_f * 1e3, 1),
                          "fwd_TBps": round(2 * n / t_f / 1e9, 2), "bwd_us": round(t_b * 1e3, 1),
                          "bwd_TBps": round(3 * n / t_b / 1e9, 2), "fwd_t_us": round(t_ft * 1e3, 1),
                          "bwd_t_us": round(t_bt * 1e3, 1), "fwd_rel_err": ef, "bwd_rel_err": eb}), flush=True)


if __name__ == "__main__":
    main()
