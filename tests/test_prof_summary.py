"""scripts/prof_summary.py --timed: only the kernels between bench.py's trace markers count."""

import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_trace(path, rows):
    cols = ["Kind", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for name, s, e in rows:
            w.writerow({"Kind": "KERNEL_DISPATCH", "Kernel_Name": name, "Start_Timestamp": s, "End_Timestamp": e})


def test_timed_summary_counts_only_the_marked_region(tmp_path):
    trace = tmp_path / "run_kernel_trace.csv"
    _write_trace(trace, [
        ("init_fill", 0, 50),                       # before the first marker: excluded
        ("dsa::dsa_profile_marker_kernel(int)", 100, 101),
        ("Cijk_gemm", 200, 300),
        ("void dsa::ln_fwd_kernel<bf16>", 300, 320),
        ("Cijk_gemm", 400, 500),
        ("dsa::dsa_profile_marker_kernel(int)", 600, 601),
        ("late_copy", 700, 900),                    # after the last marker: excluded
    ])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_summary.py"), "--timed", str(trace),
                          "title", "cmd"], capture_output=True, text=True, check=True).stdout
    assert "Total kernel time: 0.0 ms" in out  # 220 ns
    assert "wall 0.0 ms" in out
    assert "init_fill" not in out and "late_copy" not in out
    assert "| GEMM (hipBLASLt/rocBLAS) |" in out and "| 2 |" in out
    assert "dsa_profile_marker" not in out.split("| total ms |")[1]
