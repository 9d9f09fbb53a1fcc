"""NVMe/local-disk throughput sweep of the native aio engine (reference:
tests/perf/aio_bench_perf_sweep.py).  Writes then reads a pinned (page-aligned) buffer through
`aio_handle` for each (engine, block_size, queue_depth, single_submit, overlap_events,
thread_count) and prints one JSON line per point (GB/s).  O_DIRECT bypasses the page cache,
so reads measure the device, not memory.

    python scripts/aio_sweep.py --path /tmp/aio_sweep --mb 1024
"""
import argparse
import itertools
import json
import os
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_points(args):
    from deeperspeed_amd.ops.aio import AsyncIOBuilder
    aio = AsyncIOBuilder().load()
    n = args.mb * (1 << 20) // 4
    pin = torch.cuda.is_available()
    buf = torch.empty(n, dtype=torch.float32, pin_memory=pin)
    if buf.data_ptr() % 4096:
        base = torch.empty(n + 1024, dtype=torch.float32, pin_memory=pin)
        off = ((-base.data_ptr()) % 4096) // 4
        buf = base[off: off + n]
    buf.uniform_()
    os.makedirs(args.path, exist_ok=True)
    f = os.path.join(args.path, "sweep.swp")
    blocks = [int(b) << 10 for b in args.blocks.split(",")]
    qds = [int(q) for q in args.qds.split(",")]
    threads = [int(t) for t in args.threads.split(",")]
    modes = [(False, True), (True, True), (False, False)]  # (single_submit, overlap_events)
    for blk, qd, th, (ss, ov) in itertools.product(blocks, qds, threads, modes):
        h = aio.aio_handle(blk, qd, ss, ov, th)
        res = {"engine": h.get_engine(), "block_kib": blk >> 10, "queue_depth": qd, "threads": th,
               "single_submit": ss, "overlap_events": ov, "mib": args.mb}
        for op in ("write", "read"):
            best = 0.0
            for _ in range(args.reps):
                t = time.perf_counter()
                rc = h.sync_pwrite(buf, f) if op == "write" else h.sync_pread(buf, f)
                dt = time.perf_counter() - t
                assert rc == 1, f"aio {op} failed"
                best = max(best, buf.nbytes / dt / 1e9)
            res[f"{op}_GBps"] = round(best, 3)
        print(json.dumps(res), flush=True)
    os.remove(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default="/tmp/dsa_aio_sweep")
    ap.add_argument("--mb", type=int, default=1024)
    ap.add_argument("--blocks", default="128,512,1024,4096", help="KiB")
    ap.add_argument("--qds", default="1,4,16,64")
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--psync-baseline", action="store_true",
                    help="also sweep the positional-I/O engine (DSA_AIO_ENGINE=psync) in a child process")
    args = ap.parse_args()
    run_points(args)
    if args.psync_baseline and os.environ.get("DSA_AIO_ENGINE") != "psync":
        cmd = [sys.executable, os.path.abspath(__file__), "--path", args.path, "--mb", str(args.mb),
               "--blocks", args.blocks, "--qds", "1,16", "--threads", args.threads, "--reps", str(args.reps)]
        subprocess.run(cmd, env=dict(os.environ, DSA_AIO_ENGINE="psync"), check=True)


if __name__ == "__main__":
    main()
