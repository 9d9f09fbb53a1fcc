#!/bin/bash
# Round 3: block-sparse attention timing + per-kernel profile (BigBird block 64, S 8192).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 200 python scripts/bench_sparse_attn.py --unfused > gpurun_out/r3e_sparse.jsonl 2> gpurun_out/r3e_sparse.err || { tail -20 gpurun_out/r3e_sparse.err; exit 1; }
cat gpurun_out/r3e_sparse.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3e_prof -o sp --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_sparse_attn.py --iters 5 > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/r3e_prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r3e_kernel_stats.csv; head -14 gpurun_out/r3e_kernel_stats.csv | cut -c1-200
