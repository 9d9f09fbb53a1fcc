#!/bin/bash
# Round 2, run BJ: forced-sharded ZeRO-3 (world-1 RCCL) on the current tree -- bench, then kernel profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py --force-sharded > gpurun_out/r2bj_bench_sharded.json 2> gpurun_out/r2bj_bench_sharded.log || { tail -20 gpurun_out/r2bj_bench_sharded.log; exit 1; }
cut -c1-200 gpurun_out/r2bj_bench_sharded.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2bj -o sh -- python $R/bench.py --steps 2 --warmup 2 --force-sharded > $R/gpurun_out/r2bj_prof.json 2> $R/gpurun_out/r2bj_prof.log || { tail -20 $R/gpurun_out/r2bj_prof.log; exit 1; }
echo profiled
