"""Turn a rocprofv3 `*_kernel_stats.csv` into the markdown table committed under profiles/.

usage: python scripts/prof_summary.py <kernel_stats.csv> <title> <command> [note] > profiles/<name>.md
"""

import csv
import sys


def main():
    path, title, cmd = sys.argv[1:4]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    rows = list(csv.DictReader(open(path)))
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Command: `{cmd}`")
    if note:
        print(f"\n{note}")
    print(f"\nTotal kernel time: {total_ns / 1e6:.1f} ms\n")
    print("| total ms | % | calls | avg us | kernel |")
    print("|---|---|---|---|---|")
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:45]:
        name = r["Name"].replace("|", "/")
        if len(name) > 120:
            name = name[:117] + "..."
        print(f"| {float(r['TotalDurationNs']) / 1e6:.1f} | {100 * float(r['TotalDurationNs']) / total_ns:.1f} | "
              f"{r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
