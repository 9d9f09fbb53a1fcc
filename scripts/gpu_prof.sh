#!/bin/bash
# rocprofv3 kernel stats of the flagship bench (1 warmup + 1 timed step).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_head -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log; exit 1; }
tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_head -name "*stats*"
