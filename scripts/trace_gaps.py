"""Idle time of the compute stream in a rocprofv3 kernel trace, and where it sits.

    python scripts/trace_gaps.py <k_kernel_trace.csv> [--stream S] [--min-us 200] [--top 25]

Restricted to bench.py's timed region (between its dsa_profile_marker launches).  The compute
stream defaults to the one that ran the most kernel time.  For every gap between consecutive
kernels of that stream longer than --min-us it prints the gap, its offset from the start of the
timed region, the kernel before and after it, and which other streams' kernels ran inside it
(e.g. an optimizer step on a side stream, copies) -- the question "what is the forward waiting
for at the step boundary" answered from the trace.
"""

import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--stream", type=int, default=None)
    ap.add_argument("--min-us", type=float, default=200.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    marks = sorted(int(r["Start_Timestamp"]) for r in rows if "dsa_profile_marker" in r["Kernel_Name"])
    lo, hi = (marks[0], marks[-1]) if len(marks) >= 2 else (0, 1 << 62)
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if lo < s < hi and "dsa_profile_marker" not in r["Kernel_Name"]:
            ks.append((s, e, int(r["Stream_Id"]), int(r["Queue_Id"]), r["Kernel_Name"]))
    busy = defaultdict(int)
    for s, e, st, q, n in ks:
        busy[st] += e - s
    main_st = a.stream if a.stream is not None else max(busy, key=busy.get)
    wall = hi - lo if len(marks) >= 2 else max(e for _, e, *_ in ks) - min(s for s, *_ in ks)
    print(f"timed wall {wall / 1e6:.1f} ms; per-stream kernel time: "
          + ", ".join(f"stream {st}: {t / 1e6:.1f} ms" for st, t in sorted(busy.items(), key=lambda x: -x[1])))
    comp = sorted(k for k in ks if k[2] == main_st)
    others = sorted(k for k in ks if k[2] != main_st)
    gaps = []
    prev_end, prev_name = lo, "<start>"
    for s, e, st, q, n in comp:
        if s - prev_end > a.min_us * 1e3:
            gaps.append((s - prev_end, prev_end, s, prev_name, n))
        if e > prev_end:
            prev_end, prev_name = e, n
    idle = sum(g[0] for g in gaps)
    all_idle = 0
    pe = lo
    for s, e, *_ in comp:
        if s > pe:
            all_idle += s - pe
        pe = max(pe, e)
    print(f"compute stream {main_st}: busy {busy[main_st] / 1e6:.1f} ms, idle {all_idle / 1e6:.1f} ms "
          f"({100 * all_idle / wall:.1f} % of wall), of which {idle / 1e6:.1f} ms in {len(gaps)} gaps > {a.min_us:.0f} us\n")
    print("| gap ms | at ms | before | after | other streams inside the gap (ms) |")
    print("|---|---|---|---|---|")
    for g, s0, s1, pn, nn in sorted(gaps, reverse=True)[: a.top]:
        inside = defaultdict(float)
        for s, e, st, q, n in others:
            if e > s0 and s < s1:
                inside[n[:40]] += (min(e, s1) - max(s, s0)) / 1e6
        top = sorted(inside.items(), key=lambda x: -x[1])[:3]
        print(f"| {g / 1e6:.2f} | {(s0 - lo) / 1e6:.1f} | `{pn[:50]}` | `{nn[:50]}` | "
              + "; ".join(f"`{k}` {v:.1f}" for k, v in top) + " |")


if __name__ == "__main__":
    main()
