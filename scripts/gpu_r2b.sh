#!/bin/bash
# Round 2, run B: 20B forced-sharded ZeRO-3 bench on one GPU (world-1 RCCL), then a rocprofv3
# kernel-trace summary of the same path.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 420 python bench.py --steps 4 --warmup 2 --force-sharded > gpurun_out/r2b_bench_sharded.json 2> gpurun_out/r2b_bench_sharded.log || { grep -v config.py gpurun_out/r2b_bench_sharded.log | tail -30; exit 1; }
tail -c 900 gpurun_out/r2b_bench_sharded.json
grep '^\[bench\]' gpurun_out/r2b_bench_sharded.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2b -o r2b -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 2 --force-sharded > $GRAFT_REPO_ROOT/gpurun_out/r2b_prof_bench.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r2b_prof_bench.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_r2b -name '*stats*'
