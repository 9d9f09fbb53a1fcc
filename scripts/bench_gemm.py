"""Per-shape GEMM throughput of the GPT-NeoX-20B training step on one MI355X (hipBLASLt through
torch.matmul), for the three products autograd issues per nn.Linear:

    fwd   y  = x  @ W^T   [M,K] x [N,K]^T
    dgrad dx = dy @ W     [M,N] x [N,K]
    wgrad dW = dy^T @ x   [N,M] x [M,K]

    python scripts/bench_gemm.py [--tokens 8192] [--hidden 6144]
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
    ap.add_argument("--vocab", type=int, default=50432)
    a = ap.parse_args()
    M, h = a.tokens, a.hidden
    dev = torch.device("cuda")
    dt = torch.bfloat16
    shapes = {"qkv": (3 * h, h), "dense": (h, h), "h_to_4h": (4 * h, h), "4h_to_h": (h, 4 * h),
              "logits": (a.vocab, h)}
    rows = []
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=dt)
        w = torch.randn(N, K, device=dev, dtype=dt)
        dy = torch.randn(M, N, device=dev, dtype=dt)
        flop = 2.0 * M * N * K
        for op, fn in (("fwd", lambda: torch.matmul(x, w.t())),
                       ("dgrad", lambda: torch.matmul(dy, w)),
                       ("wgrad", lambda: torch.matmul(dy.t(), x))):
            ms = bench(fn)
            rows.append({"gemm": name, "op": op, "M": M, "N": N, "K": K, "ms": round(ms, 3),
                         "tflops": round(flop / ms / 1e9, 1)})
            print(json.dumps(rows[-1]), flush=True)
        del x, w, dy
    tot_ms = sum(r["ms"] for r in rows if r["gemm"] != "logits")
    tot_fl = sum(2.0 * r["M"] * r["N"] * r["K"] for r in rows if r["gemm"] != "logits")
    print(json.dumps({"layer_gemm_ms": round(tot_ms, 3), "layer_tflops": round(tot_fl / tot_ms / 1e9, 1)}))


if __name__ == "__main__":
    main()
