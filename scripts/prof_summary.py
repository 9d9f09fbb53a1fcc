"""Turn a rocprofv3 kernel trace into the markdown table committed under profiles/.

Accepts either a `*_kernel_stats.csv` (--output-format csv) or the default SQLite output
(`*_results.db`, aggregated from its `kernels` view).  Besides the per-kernel table it
prints a category breakdown (hipBLASLt GEMMs, RCCL, own HIP kernels, torch elementwise,
fills / copies) so the non-GEMM share can be tracked across rounds.

usage: python scripts/prof_summary.py [--timed] <stats.csv|results.db|kernel_trace.csv> <title> <command> [note]
           > profiles/<name>.md   (--timed: a kernel_trace.csv restricted to the timed steps)
"""

import csv
import sqlite3
import sys
from collections import defaultdict


def load_timed(path):
    """[(name, calls, total_ns)] of the kernels between the dsa_profile_marker launches (tag 1 /
    tag 2, written by bench.py around its timed steps) in a rocprofv3 `*_kernel_trace.csv`."""
    rows = list(csv.DictReader(open(path)))
    marks = sorted(int(r["Start_Timestamp"]) for r in rows if "dsa_profile_marker" in r["Kernel_Name"])
    if len(marks) < 2:
        raise SystemExit("no timed-region markers in the trace (bench.py launches them on the GPU)")
    lo, hi = marks[0], marks[-1]
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        s, e, n = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]
        if lo < s < hi and "dsa_profile_marker" not in n:
            agg[n][0] += 1
            agg[n][1] += e - s
    return [(n, k, t) for n, (k, t) in agg.items()], (hi - lo)


def load(path):
    """[(name, calls, total_ns)]"""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select name, count(*), sum(duration) from kernels group by name").fetchall()
        return [(n, int(k), float(t)) for n, k, t in rows]
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))]


def category(name):
    n = name.lower()
    if "cijk_" in n or "gemm" in n and "dsa::" not in n:
        return "GEMM (hipBLASLt/rocBLAS)"
    if "nccl" in n or "rccl" in n:
        return "RCCL collectives"
    if "dsa::fa::" in n:
        return "flash attention (own HIP)"
    if "dsa::" in n:
        return "other own HIP kernels"
    if "fill" in n:
        return "fills / memset"
    if "copy" in n or "memcpy" in n:
        return "copies"
    if "at::native" in n:
        return "torch elementwise / reductions"
    return "other"


def main():
    args = [a for a in sys.argv[1:] if a != "--timed"]
    timed = "--timed" in sys.argv[1:]
    path, title, cmd = args[:3]
    note = args[3] if len(args) > 3 else ""
    wall = None
    if timed:  # path is a *_kernel_trace.csv: only the kernels of the timed steps
        rows, wall = load_timed(path)
    else:
        rows = load(path)
    total_ns = sum(t for _, _, t in rows)
    print(f"# {title}\n")
    print(f"Command: `{cmd}`")
    if note:
        print(f"\n{note}")
    print(f"\nTotal kernel time: {total_ns / 1e6:.1f} ms" +
          (f" (timed steps only, between bench.py's trace markers; wall {wall / 1e6:.1f} ms)" if wall else "") + "\n")
    cats = defaultdict(lambda: [0, 0.0])
    for n, k, t in rows:
        c = cats[category(n)]
        c[0] += k
        c[1] += t
    print("| category | total ms | % | calls |")
    print("|---|---|---|---|")
    for name, (k, t) in sorted(cats.items(), key=lambda kv: -kv[1][1]):
        print(f"| {name} | {t / 1e6:.1f} | {100 * t / total_ns:.1f} | {k} |")
    print("\n| total ms | % | calls | avg us | kernel |")
    print("|---|---|---|---|---|")
    rows.sort(key=lambda r: -r[2])
    for n, k, t in rows[:45]:
        name = n.replace("|", "/")
        if len(name) > 120:
            name = name[:117] + "..."
        print(f"| {t / 1e6:.1f} | {100 * t / total_ns:.1f} | {k} | {t / k / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
