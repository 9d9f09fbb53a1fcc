"""Which weight storage layout gives hipBLASLt its fastest kernels for the GPT-NeoX-20B GEMMs?

Per nn.Linear (x [M,K], dy [M,N]) and weight storage:
    W  [N,K] (torch default): fwd x @ W^T,  dgrad dy @ W,    wgrad dy^T @ x  (-> [N,K])
    Wt [K,N] (transposed):    fwd x @ Wt,   dgrad dy @ Wt^T, wgrad x^T @ dy  (-> [K,N])
wgrad is timed both as a fresh product and accumulated in place (addmm_, beta = 1), as the
framework's fused-wgrad linear issues it.  Also times the rocBLAS backend for comparison.

    python scripts/bench_gemm_layouts.py --tokens 8192
"""

import argparse
import json

import torch


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--hidden", type=int, default=6144)
    ap.add_argument("--backends", type=str, default="cublaslt,cublas")
    a = ap.parse_args()
    M, h = a.tokens, a.hidden
    dev = torch.device("cuda")
    dt = torch.bfloat16
    shapes = {"qkv": (3 * h, h), "dense": (h, h), "h_to_4h": (4 * h, h), "4h_to_h": (h, 4 * h)}
    for be in a.backends.split(","):
        try:
            torch.backends.cuda.preferred_blas_library(be)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"backend": be, "error": str(e)}))
            continue
        tot = {}
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=dt)
            dy = torch.randn(M, N, device=dev, dtype=dt)
            W = torch.randn(N, K, device=dev, dtype=dt)
            Wt = W.t().contiguous()
            gW = torch.zeros(N, K, device=dev, dtype=dt)
            gWt = torch.zeros(K, N, device=dev, dtype=dt)
            flop = 2.0 * M * N * K
            ops = {
                "W.fwd": lambda: x @ W.t(), "W.dgrad": lambda: dy @ W, "W.wgrad": lambda: dy.t() @ x,
                "W.wgrad_acc": lambda: gW.addmm_(dy.t(), x),
                "Wt.fwd": lambda: x @ Wt, "Wt.dgrad": lambda: dy @ Wt.t(), "Wt.wgrad": lambda: x.t() @ dy,
                "Wt.wgrad_acc": lambda: gWt.addmm_(x.t(), dy),
            }
            for op, fn in ops.items():
                ms = bench(fn)
                tot[op] = tot.get(op, 0.0) + ms
                print(json.dumps({"backend": be, "gemm": name, "op": op, "M": M, "N": N, "K": K, "ms": round(ms, 3),
                                  "tflops": round(flop / ms / 1e9, 1)}), flush=True)
            del x, dy, W, Wt, gW, gWt
        print(json.dumps({"backend": be, "layer_total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
