"""Tune the GPT-NeoX GEMMs with PyTorch TunableOp (hipBLASLt + rocBLAS solution search) and
report default vs tuned time per shape.

The NeoX training step issues, per nn.Linear (x:[M,K], W:[N,K], bias:[N]):
    fwd   y  = x @ W^T + b   (addmm, hipBLASLt bias epilogue)
    dgrad dx = dy @ W
    wgrad dW = dy^T @ x
The tuned table is written to --out (TunableOp CSV); `deeperspeed_amd.ops.gemm_tuning`
loads it at engine start when the file exists for this device.

    python scripts/tune_gemm.py --out deeperspeed_amd/ops/tuned/gemm_gfx950.csv
"""

import argparse
import json
import os

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


def ops_for(M, N, K, dev, dt):
    x = torch.randn(M, K, device=dev, dtype=dt)
    w = torch.randn(N, K, device=dev, dtype=dt)
    b = torch.randn(N, device=dev, dtype=dt)
    dy = torch.randn(M, N, device=dev, dtype=dt)
    return {"fwd": lambda: torch.nn.functional.linear(x, w, b),
            "fwd_nobias": lambda: torch.nn.functional.linear(x, w),
            "dgrad": lambda: torch.matmul(dy, w),
            "wgrad": lambda: torch.matmul(dy.t(), x)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[8192])
    ap.add_argument("--hidden", type=int, default=6144)
    ap.add_argument("--vocab", type=int, default=50432)
    ap.add_argument("--out", type=str, default="gpurun_out/tunableop_gfx950.csv")
    ap.add_argument("--max-ms", type=int, default=400, help="tuning budget per GEMM")
    a = ap.parse_args()
    dev = torch.device("cuda")
    dt = torch.bfloat16
    h = a.hidden
    shapes = {"qkv": (3 * h, h), "dense": (h, h), "h_to_4h": (4 * h, h), "4h_to_h": (h, 4 * h),
              "logits": (a.vocab, h)}
    default = {}
    for M in a.tokens:
        for name, (N, K) in shapes.items():
            for op, fn in ops_for(M, N, K, dev, dt).items():
                default[(M, name, op)] = bench(fn)
            torch.cuda.empty_cache()
    import torch.cuda.tunable as tun
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    tun.set_filename(a.out, insert_device_ordinal=False)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_max_tuning_iterations(100)
    rows = []
    for M in a.tokens:
        for name, (N, K) in shapes.items():
            for op, fn in ops_for(M, N, K, dev, dt).items():
                fn()  # tunes on first call
                ms = bench(fn)
                d = default[(M, name, op)]
                flop = 2.0 * M * N * K
                rows.append({"M": M, "gemm": name, "op": op, "N": N, "K": K, "default_ms": round(d, 3),
                             "tuned_ms": round(ms, 3), "default_tflops": round(flop / d / 1e9, 1),
                             "tuned_tflops": round(flop / ms / 1e9, 1)})
                print(json.dumps(rows[-1]), flush=True)
            torch.cuda.empty_cache()
    tun.write_file()
    td = sum(r["default_ms"] for r in rows if r["op"] != "fwd_nobias")
    tt = sum(r["tuned_ms"] for r in rows if r["op"] != "fwd_nobias")
    print(json.dumps({"sum_default_ms": round(td, 3), "sum_tuned_ms": round(tt, 3), "file": a.out}))


if __name__ == "__main__":
    main()
