"""Layer-batched weight-gradient GEMMs of BERT-Large (ops/wgrad_batch.py): torch.baddbmm_ (hipBLASLt's
first heuristic answer) against the extension's timed strided-batched hipBLASLt call
(`gemm_lt_batched`: heuristic top-16 + table-registered names) and an exhaustive sweep of every
solution for the same strided-batched problem (NT, as the slabs hold the operands, and TN, the
layout transposed operands would allow).

    python scripts/bench_wgrad_lt.py [--layers 24] [--tokens 8192] [--sweep] > out.jsonl
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deeperspeed_amd.ops import native  # noqa: E402

SHAPES = {"qkv": (3072, 1024), "attn_out": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096)}  # (N, K)


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
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--sweep", action="store_true")
    args = ap.parse_args()
    ops = native.hip_ops()
    L, M = args.layers, args.tokens
    dev = torch.device("cuda")
    for name, (N, K) in SHAPES.items():
        dy = torch.randn(L, M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(L, M, K, device=dev, dtype=torch.bfloat16)
        gw = torch.zeros(L, N, K, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * L * M * N * K
        t_torch = timed(lambda: gw.baddbmm_(dy.transpose(1, 2), x))
        gw2 = torch.zeros_like(gw)
        t_lt = timed(lambda: ops.gemm_lt_batched(dy, x, True, False, gw2, True))
        # numerics: one accumulate from zero against fp32
        a = torch.zeros_like(gw)
        ops.gemm_lt_batched(dy, x, True, False, a, True)
        ref = torch.bmm(dy.float().transpose(1, 2), x.float())
        err = ((a.float() - ref).abs().max() / ref.abs().max()).item()
        rec = {"linear": name, "L": L, "M": M, "N": N, "K": K, "baddbmm_ms": round(t_torch, 3),
               "baddbmm_tflops": round(flops / t_torch / 1e9, 1), "lt_batched_ms": round(t_lt, 3),
               "lt_batched_tflops": round(flops / t_lt / 1e9, 1), "lt_rel_err": err}
        if args.sweep:
            # lt_sweep kind 2 (NT, operands as the slabs hold them) / 3 (TN, x^T and dy^T stored)
            # of row-major (tokens M, out N, in K): the [N, K] weight gradient, accumulated
            for kind, lay in ((2, "NT"), (3, "TN")):
                heur_ms, n_all, n_timed, top = ops.lt_sweep(kind, M, N, K, False, 4, L)
                rec[f"sweep_{lay}"] = {"heuristic_tflops": round(flops / heur_ms / 1e9, 1) if heur_ms > 0 else None,
                                       "algos": n_all, "timed": n_timed,
                                       "top": [{"tflops": round(flops / ms / 1e9, 1), "sol": sol, "kernel": kn[:100]}
                                               for ms, sol, kn in top]}
        print(json.dumps(rec), flush=True)
        del dy, x, gw, gw2, a, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
