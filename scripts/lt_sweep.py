"""Exhaustive hipBLASLt sweep with the library this framework actually runs on.

torch bundles its own hipBLASLt build and the HIP extension binds to it, so the sweep runs inside
the extension (`lt_sweep` in ops/csrc/gemm_lt.cpp) rather than as a program linked against
/opt/rocm (scripts/lt_sweep.cpp: same sweep, /opt/rocm's build; solution sets differ).

    python scripts/lt_sweep.py out.jsonl fwdb:8192:18432:6144 dgrad:8192:18432:6144 ...

layouts (row-major): fwd / fwdb (forward, + bias epilogue), dgrad (NN), wgrad (NT, accumulate),
wgradT (TN after operand transposes, accumulate).  One JSON line per problem, the format
scripts/make_lt_table.py reads.
"""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deeperspeed_amd.ops import lt_tune, native  # noqa: E402

KINDS = {"fwd": 0, "fwdb": 0, "dgrad": 1, "wgrad": 2, "wgradT": 3}


def main(out, specs):
    ops = native.hip_ops()
    lib = ops.lt_library()
    with open(out, "a") as f:
        for spec in specs:
            lay, M, N, K = spec.split(":")
            M, N, K = int(M), int(N), int(K)
            bias = lay == "fwdb"
            t0 = time.time()
            heur_ms, n_all, n_timed, top = ops.lt_sweep(KINDS[lay], M, N, K, bias, 6)
            flops = 2.0 * M * N * K
            kind = "fwd" if lay == "fwdb" else lay
            c = lt_tune.key(kind, M, N, K, bias)
            rec = {"layout": kind + ("+bias" if bias else ""), "M": M, "N": N, "K": K, "algos": n_all,
                   "supported": n_timed, "heuristic_tflops": round(flops / heur_ms / 1e9, 1) if heur_ms > 0 else None,
                   "col": dict(zip(("ta", "tb", "m", "n", "k", "epi", "beta"), c)),
                   "top": [{"tflops": round(flops / ms / 1e9, 1), "sol": sol, "kernel": kn[:120]} for ms, sol, kn in top],
                   "library": lib, "sweep_s": round(time.time() - t0, 1)}
            f.write(json.dumps(rec) + "\n")
            f.flush()
            best = rec["top"][0]["tflops"] if rec["top"] else None
            print(f"{rec['layout']} {M}x{N}x{K}: heuristic {rec['heuristic_tflops']} best {best} TF/s "
                  f"({n_timed} timed, {rec['sweep_s']} s)", flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
