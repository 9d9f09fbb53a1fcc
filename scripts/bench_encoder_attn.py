"""Encoder (BERT) attention micro-benchmark: the fused QKV-layout flash kernels with and without
the key-padding bias and the in-kernel dropout, next to the plain head-major non-causal flash
kernel, at the BERT-Large shapes (D 64).  One JSON line per variant (fwd / bwd ms, TFLOP/s at
4*B*H*S^2*D forward FLOPs, 2.5x that backward)."""

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
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="16x512,64x128", help="BxS list")
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    H, D = a.H, a.D
    for shp in a.shapes.split(","):
        B, S = (int(x) for x in shp.split("x"))
        flops = 4.0 * B * H * S * S * D
        qkv = torch.randn(B, S, 3 * H * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        do = torch.randn(B, S, H * D, device=dev, dtype=torch.bfloat16)
        mask = torch.zeros(B, S, device=dev)
        mask[:, S - S // 8:] = -10000.0  # padded tail
        g = torch.Generator().manual_seed(0)
        variants = [
            ("qkv bias+dropout (BERT path)", lambda: native.flash_attention_qkv(qkv, H, mask, D ** -0.5, 0.1, True, g)),
            ("qkv bias only", lambda: native.flash_attention_qkv(qkv, H, mask, D ** -0.5, 0.0, True, g)),
            ("qkv no bias, no dropout", lambda: native.flash_attention_qkv(qkv, H, None, D ** -0.5, 0.0, True, g)),
        ]
        q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
        dob = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16)
        variants.append(("head-major non-causal", lambda: native.flash_attention(q, k, v, False, D ** -0.5)))
        for name, fn in variants:
            tf = timeit(fn, a.iters)
            o = fn()
            ins = (q, k, v) if name.startswith("head") else (qkv,)
            gout = dob if name.startswith("head") else do
            tb = timeit(lambda: torch.autograd.grad(o, ins, gout, retain_graph=True), a.iters)
            print(json.dumps({"variant": name, "B": B, "S": S, "H": H, "D": D, "fwd_ms": round(tf * 1e3, 4),
                              "bwd_ms": round(tb * 1e3, 4), "fwd_tflops": round(flops / tf / 1e12, 1),
                              "bwd_tflops": round(2.5 * flops / tb / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
