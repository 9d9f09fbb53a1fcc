#!/bin/bash
# Round 3: 20B N=1 bench on the current tree, same-box A/B against the round-2 kernels
# (row-per-thread rotary, dK/dV v2 + separate Delta kernel), and a kernel profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 420 python bench.py --steps 8 --warmup 4 > gpurun_out/r3h_bench_n1.json 2> gpurun_out/r3h_bench_n1.log || { tail -30 gpurun_out/r3h_bench_n1.log; exit 1; }
cat gpurun_out/r3h_bench_n1.json
DSA_ROTARY_TILED=0 DSA_FA_DKDV=2 DSA_FA_FUSED_DELTA=0 timeout -k 10 420 python bench.py --steps 8 --warmup 4 > gpurun_out/r3h_bench_n1_r2kernels.json 2> gpurun_out/r3h_bench_n1_r2kernels.log || { tail -30 gpurun_out/r3h_bench_n1_r2kernels.log; exit 1; }
cat gpurun_out/r3h_bench_n1_r2kernels.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3h_prof -o neox --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 2 > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/r3h_prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r3h_kernel_stats.csv; echo profiled
