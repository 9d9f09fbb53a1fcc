"""Build deeperspeed_amd/ops/lt_table.json from lt_sweep JSON lines (scripts/lt_sweep.cpp).

    python scripts/make_lt_table.py profiles/r4i_lt_sweep*.jsonl

Each entry keeps the column-major problem, the fastest solutions by hipBLASLt solution name (they join the
heuristic candidates that ops/csrc/gemm_lt.cpp times on first use) and the best / heuristic
rates measured by the sweep (ops/lt_tune.py's NT-vs-TN weight-gradient choice reads them).
"""

import json
import os
import sys

OUT = os.path.join(os.path.dirname(__file__), "..", "deeperspeed_amd", "ops", "lt_table.json")


def col_of(layout, M, N, K):
    """Column-major problem of a row-major layout record (ops/lt_tune.py: key)."""
    kind, _, extra = layout.partition("+")
    ta, tb, m, n, k, beta = {"fwd": (1, 0, N, M, K, 0), "dgrad": (0, 0, K, M, N, 0),
                             "wgrad": (0, 1, K, N, M, 1), "wgradT": (1, 0, K, N, M, 1)}[kind]
    return {"ta": ta, "tb": tb, "m": m, "n": n, "k": k, "epi": 4 if extra == "bias" else 1, "beta": beta}


def main(paths):
    entries = {}
    for p in paths:
        with open(p) as f:
            for line in f:
                line = line.strip()
                if not line.startswith("{"):
                    continue
                r = json.loads(line)
                if not r.get("top"):
                    continue
                c = r.get("col") or col_of(r["layout"], r["M"], r["N"], r["K"])
                k = (c["ta"], c["tb"], c["m"], c["n"], c["k"], c["epi"], c["beta"])
                e = {"layout": r["layout"], "M": r["M"], "N": r["N"], "K": r["K"], "col": c,
                     "names": [t["sol"] for t in r["top"] if t.get("sol")], "tflops": r["top"][0]["tflops"],
                     "heuristic_tflops": r["heuristic_tflops"], "kernel": r["top"][0]["kernel"], "source": p}
                old = entries.get(k)
                if old is None or e["tflops"] > old["tflops"]:
                    if old is not None:
                        e["names"] += [n for n in old["names"] if n not in e["names"]]
                    entries[k] = e
    data = {"about": "fastest hipBLASLt solutions per GEMM problem on MI355X (gfx950), from scripts/lt_sweep.cpp; "
                     "read by deeperspeed_amd/ops/lt_tune.py",
            "entries": sorted(entries.values(), key=lambda e: (e["M"], e["N"], e["K"], e["layout"]))}
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1)
    print(f"{len(entries)} entries -> {os.path.normpath(OUT)}")


if __name__ == "__main__":
    main(sys.argv[1:])
