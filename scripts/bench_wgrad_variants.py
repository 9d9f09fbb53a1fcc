"""Weight/input-gradient GEMM formulations for the GPT-NeoX-20B linears (hipBLASLt via torch).

Row-major notation; "NT" = both operands contiguous along the reduction dim (the fastest
hipBLASLt kernels on gfx950 in scripts/bench_gemm_layouts.py).

    wgrad  dW[N,K] = dy^T x (reduction over the M tokens)
      tn       : dy.t() @ x                                  (autograd default)
      nt_T     : transpose dy and x explicitly, then NT      (includes both transposes)
      nn_dyT   : dy.t().contiguous() @ x
      nn_xT    : dy.t() @ x.t().contiguous().t()
    dgrad  dx[M,K] = dy W
      nn       : dy @ W                                      (autograd default)
      nt_T     : dy @ W.t().contiguous().t()                 (includes the weight transpose)

    python scripts/bench_wgrad_variants.py
"""

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
    M, h = 8192, 6144
    dev, dt = torch.device("cuda"), torch.bfloat16
    shapes = {"qkv": (3 * h, h), "dense": (h, h), "h_to_4h": (4 * h, h), "4h_to_h": (h, 4 * h)}
    tot = {}
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=dt)
        dy = torch.randn(M, N, device=dev, dtype=dt)
        W = torch.randn(N, K, device=dev, dtype=dt)
        flop = 2.0 * M * N * K
        ops = {
            "wgrad.tn": lambda: dy.t() @ x,
            "wgrad.nt_T": lambda: dy.t().contiguous() @ x.t().contiguous().t(),
            "wgrad.nn_dyT": lambda: dy.t().contiguous() @ x,
            "wgrad.nn_xT": lambda: dy.t() @ x.t().contiguous().t(),
            "transpose.x": lambda: x.t().contiguous(),
            "transpose.dy": lambda: dy.t().contiguous(),
            "dgrad.nn": lambda: dy @ W,
            "dgrad.nt_T": lambda: dy @ W.t().contiguous().t(),
            "transpose.W": lambda: W.t().contiguous(),
        }
        for op, fn in ops.items():
            ms = bench(fn)
            tot[op] = tot.get(op, 0.0) + ms
            print(json.dumps({"gemm": name, "op": op, "ms": round(ms, 3),
                              "tflops": None if op.startswith("transpose") else round(flop / ms / 1e9, 1)}), flush=True)
        del x, dy, W
    print(json.dumps({"layer_total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
