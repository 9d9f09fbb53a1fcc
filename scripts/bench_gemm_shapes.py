"""GEMM variants at the transformer shapes: torch (hipBLASLt default heuristic) vs the autotuned
hipBLASLt wrapper (`_hip_ops.gemm_lt`), for the forward, input-gradient and weight-gradient
products of each linear, in the layouts the framework can produce.

    python scripts/bench_gemm_shapes.py --model bert-large --tokens 8192
    python scripts/bench_gemm_shapes.py --model neox20b --tokens 8192
Prints one JSON line per (linear, product, variant) with ms and TFLOP/s.
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: [(linear, in, out)]
    "bert-large": [("qkv", 1024, 3072), ("attn_out", 1024, 1024), ("fc1", 1024, 4096), ("fc2", 4096, 1024)],
    "bert-base": [("qkv", 768, 2304), ("attn_out", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)],
    "neox20b": [("qkv", 6144, 18432), ("dense", 6144, 6144), ("fc1", 6144, 24576), ("fc2", 24576, 6144)],
}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large")
    ap.add_argument("--tokens", type=int, default=8192)
    args = ap.parse_args()
    from deeperspeed_amd.ops import native
    ops = native.hip_ops()
    dev = torch.device("cuda")
    M = args.tokens
    for name, fin, fout in SHAPES[args.model]:
        x = torch.randn(M, fin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(fout, fin, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(M, fout, device=dev, dtype=torch.bfloat16)
        wt = w.t().contiguous()
        xt, dyt = x.t().contiguous(), dy.t().contiguous()
        gw = torch.zeros(fout, fin, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * M * fin * fout
        variants = {
            ("fwd", "torch x@w^T"): lambda: torch.nn.functional.linear(x, w),
            ("fwd", "lt x@w^T"): lambda: ops.gemm_lt(x, w, False, True),
            ("fwd", "lt x@wT"): lambda: ops.gemm_lt(x, wt, False, False),
            ("dgrad", "torch dy@w"): lambda: dy @ w,
            ("dgrad", "torch dy@(wT)^T"): lambda: dy @ wt.t(),
            ("dgrad", "lt dy@w"): lambda: ops.gemm_lt(dy, w, False, False),
            ("dgrad", "lt dy@(wT)^T"): lambda: ops.gemm_lt(dy, wt, False, True),
            ("wgrad", "torch addmm dy^T x"): lambda: gw.addmm_(dy.t(), x),
            ("wgrad", "torch addmm dyT xT^T"): lambda: gw.addmm_(dyt, xt.t()),
            ("wgrad", "lt acc dy^T x"): lambda: ops.gemm_lt(dy, x, True, False, gw, True),
            ("wgrad", "lt acc dyT xT^T"): lambda: ops.gemm_lt(dyt, xt, False, True, gw, True),
            ("wgrad", "bmm split2 + sum"): lambda: gw.add_(torch.bmm(dy.view(2, M // 2, fout).transpose(1, 2),
                                                                      x.view(2, M // 2, fin)).sum(0)),
            ("wgrad", "bmm split4 + sum"): lambda: gw.add_(torch.bmm(dy.view(4, M // 4, fout).transpose(1, 2),
                                                                      x.view(4, M // 4, fin)).sum(0)),
            ("wgrad", "lt split2 acc"): lambda: [ops.gemm_lt(dy[i * (M // 2):(i + 1) * (M // 2)],
                                                             x[i * (M // 2):(i + 1) * (M // 2)], True, False, gw, True)
                                                 for i in range(2)],
            ("transpose", "x and dy (HIP)"): lambda: (native.transpose2d(x), native.transpose2d(dy)),
        }
        ref = {"fwd": torch.nn.functional.linear(x.float(), w.float()), "dgrad": dy.float() @ w.float()}
        for (prod, var), fn in variants.items():
            err = None
            if prod in ref:
                err = float((fn().float() - ref[prod]).abs().max() / ref[prod].abs().max())
            ms = timeit(fn)
            tf = None if prod == "transpose" else round(flops / ms / 1e9, 1)
            print(json.dumps({"model": args.model, "tokens": M, "linear": name, "in": fin, "out": fout, "product": prod,
                              "variant": var, "ms": round(ms, 4), "tflops": tf,
                              "rel_err": None if err is None else round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
