"""hipBLASLt epilogue fusion at the GPT-NeoX-20B MLP shapes (M tokens x H 6144 x I 24576), vs
the current composition (hipBLASLt GEMM + separate HIP elementwise kernel).  Numerics vs an
fp32 PyTorch reference, times by HIP events.  One JSON line per variant.

    python scripts/bench_gemm_epilogue.py --tokens 8192
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--hidden", type=int, default=6144)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from deeperspeed_amd.ops import native
    from deeperspeed_amd.ops.linear import input_grad
    ops = native.hip_ops()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    M, H = a.tokens, a.hidden
    I = 4 * H
    bf = torch.bfloat16
    x = torch.randn(M, H, device=dev, dtype=bf)
    w1 = torch.randn(I, H, device=dev, dtype=bf) * 0.02
    b1 = torch.randn(I, device=dev, dtype=bf) * 0.1
    w2 = torch.randn(H, I, device=dev, dtype=bf) * 0.02
    b2 = torch.randn(H, device=dev, dtype=bf) * 0.1
    res = torch.randn(M, H, device=dev, dtype=bf)
    dy = torch.randn(M, H, device=dev, dtype=bf)

    def t(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    out = []
    # --- fc1 + bias + GeLU(tanh), keeping the pre-activation
    base = lambda: native.hip_ops().bias_gelu_fwd(F.linear(x, w1), b1, True)
    fused = lambda: ops.linear_lt(x, w1, b1, None, True, None)
    ref = F.gelu(x.float() @ w1.float().t() + b1.float(), approximate="tanh")
    y = fused()
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    plain = lambda: F.linear(x, w1)
    fl = 2 * M * H * I
    tb, tf = t(base), t(fused)
    tp = t(plain)
    out.append({"op": "fc1+bias+gelu (GELU_BIAS epilogue)", "ms_separate": round(tb, 3), "ms_fused": round(tf, 3),
                "ms_plain_gemm": round(tp, 3), "tflops_fused": round(fl / tf / 1e9, 1), "rel_err": err})
    # --- fc2 + bias + residual
    h = torch.randn(M, I, device=dev, dtype=bf) * 0.5
    base2 = lambda: F.linear(h, w2, b2) + res
    fused2 = lambda: ops.linear_lt(h, w2, b2, res, False, None)
    ref2 = h.float() @ w2.float().t() + b2.float() + res.float()
    err2 = ((fused2().float() - ref2).abs().max() / ref2.abs().max()).item()
    tb, tf = t(base2), t(fused2)
    out.append({"op": "fc2+bias+residual", "ms_separate": round(tb, 3), "ms_fused": round(tf, 3),
                "tflops_fused": round(fl / tf / 1e9, 1), "rel_err": err2})
    for r in out:
        r.update(M=M, H=H, I=I)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
