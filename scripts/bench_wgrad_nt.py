"""Weight-gradient formulations for the GPT-NeoX-20B linears on MI355X (hipBLASLt via torch + HIP
transpose, ops/csrc/kernels/transpose.hip).

    tm   : gw.addmm_(dy.t(), x); b.add_(dy.sum(0))                (token-major operands)
    nt   : dyT = transpose2d(dy, b, accum) ; xT = transpose2d(x) ; gw.addmm_(dyT, xT.t())
    tr.* : the transposes alone (with and without the fused bias column sum)

    python scripts/bench_wgrad_nt.py [--tokens 8192 16384]
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
    from deeperspeed_amd.ops import native
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[8192, 16384])
    args = ap.parse_args()
    h = 6144
    dev, dt = torch.device("cuda"), torch.bfloat16
    shapes = {"qkv": (3 * h, h), "dense": (h, h), "h_to_4h": (4 * h, h), "4h_to_h": (h, 4 * h)}
    for M in args.tokens:
        tot = {}
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=dt)
            dy = torch.randn(M, N, device=dev, dtype=dt)
            gw = torch.zeros(N, K, device=dev, dtype=dt)
            gb = torch.zeros(N, device=dev, dtype=dt)
            flop = 2.0 * M * N * K

            def tm():
                gw.addmm_(dy.t(), x)
                gb.add_(dy.sum(0))

            def nt():
                dyt = native.transpose2d(dy, gb, accum=True)
                xt = native.transpose2d(x)
                gw.addmm_(dyt, xt.t())

            dyt0, xt0 = native.transpose2d(dy), native.transpose2d(x)
            ops = {"tm": tm, "nt": nt, "nt.gemm_only": lambda: gw.addmm_(dyt0, xt0.t()),
                   "tr.dy+bias": lambda: native.transpose2d(dy, gb, accum=True),
                   "tr.x": lambda: native.transpose2d(x), "torch.tr.x": lambda: x.t().contiguous()}
            for op, fn in ops.items():
                ms = bench(fn)
                tot[op] = tot.get(op, 0.0) + ms
                rec = {"M": M, "gemm": name, "op": op, "ms": round(ms, 3)}
                if op.startswith("tr.") or op.startswith("torch.tr"):
                    nbytes = 2 * 2 * (M * (N if "dy" in op else K))
                    rec["TB/s"] = round(nbytes / ms / 1e9, 2)
                else:
                    rec["tflops"] = round(flop / ms / 1e9, 1)
                print(json.dumps(rec), flush=True)
            del x, dy, gw, gb, dyt0, xt0
        print(json.dumps({"M": M, "layer_total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
