"""CPU Adam (ops/adam/cpu_adam.py over ops/csrc/cpu/cpu_adam.cpp, AVX-512/AVX2) against
torch.optim.Adam on the same host tensors -- BASELINE.md row 14 (the reference's DeepSpeedCPUAdam:
5.1-6.5x torch's Adam at 1-10 B parameters on AVX-512 hosts).

    python scripts/bench_cpu_adam.py [--params 2.5e8] [--steps 5] [--threads N]

Prints one JSON line: ms per step for both, the speedup, and the max abs difference of the updated
parameters after the timed steps (both optimizers start from the same values).
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=float, default=2.5e8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    if args.threads:
        torch.set_num_threads(args.threads)
    from deeperspeed_amd.ops.adam import DeepSpeedCPUAdam
    n = int(args.params)
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * 1e-2 for _ in range(2)]
    res = {}
    finals = {}
    for name in ("torch", "cpu_adam"):
        p = torch.nn.Parameter(p0.clone())
        if name == "torch":
            opt = torch.optim.Adam([p], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)
        else:
            opt = DeepSpeedCPUAdam([p], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw_mode=False)
        p.grad = grads[0]
        opt.step()  # warm-up (state allocation)
        t0 = time.perf_counter()
        for i in range(args.steps):
            p.grad = grads[(i + 1) % 2]
            opt.step()
        res[name] = (time.perf_counter() - t0) / args.steps * 1e3
        finals[name] = p.detach().clone()
        del opt, p
    out = {"params": n, "threads": torch.get_num_threads(), "torch_adam_ms": round(res["torch"], 1),
           "cpu_adam_ms": round(res["cpu_adam"], 1), "speedup": round(res["torch"] / res["cpu_adam"], 2),
           "max_abs_diff": float((finals["torch"] - finals["cpu_adam"]).abs().max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
