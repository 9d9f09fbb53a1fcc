"""Attention micro-benchmark: fused HIP flash kernel vs the materialised path
(GEMM -> HIP softmax -> GEMM) at GPT-NeoX shapes.  Prints one JSON line per config."""

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    from deeperspeed_amd.ops import native
    from deeperspeed_amd.ops.attention import attention
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--D", type=int, nargs="+", default=[96, 128, 64])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--flash-only", action="store_true", help="skip the unfused path (profiling runs)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for D in a.D:
        q, k, v = (torch.randn(a.B, a.H, a.S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
                   for _ in range(3))
        do = torch.randn_like(q)
        flops_f = 4 * a.B * a.H * a.S * a.S * D / 2  # causal
        res = {"B": a.B, "H": a.H, "S": a.S, "D": D}
        paths = [("flash", lambda: native.flash_attention(q, k, v, True, D ** -0.5)),
                 ("unfused", lambda: attention(q, k, v, causal=True, softmax_scale=D ** -0.5, use_flash=False))]
        for name, fn in paths[:1] if a.flash_only else paths:
            tf = timeit(lambda: fn(), a.iters)
            o = fn()
            tb = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), a.iters)
            res[f"{name}_fwd_ms"] = round(tf * 1e3, 3)
            res[f"{name}_bwd_ms"] = round(tb * 1e3, 3)
            res[f"{name}_fwd_tflops"] = round(flops_f / tf / 1e12, 1)
            res[f"{name}_bwd_tflops"] = round(2.5 * flops_f / tb / 1e12, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
