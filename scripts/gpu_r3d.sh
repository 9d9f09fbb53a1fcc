#!/bin/bash
# Round 3: flash backward with Delta fused into the dQ kernel (dQ first, then dK/dV v3).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_neox_stash_gpu.py -m gpu -x -q -k "flash or attention or neox" --timeout 120 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1 || { tail -40 gpurun_out/r3d_tests.log; exit 1; }
tail -1 gpurun_out/r3d_tests.log
for v in "3 0" "3 1" "2 1" "3 1"; do
  set -- $v
  DSA_FA_DKDV=$1 DSA_FA_FUSED_DELTA=$2 timeout -k 10 120 python scripts/bench_attn.py --D 96 --flash-only --iters 30 > gpurun_out/r3d_attn.json 2>gpurun_out/r3d_attn.err || { tail -20 gpurun_out/r3d_attn.err; exit 1; }
  echo "dkdv=$1 fused_delta=$2 $(cat gpurun_out/r3d_attn.json)"
done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3d_prof -o fa -- python3 $GRAFT_REPO_ROOT/scripts/bench_attn.py --D 96 --flash-only --iters 10 > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/r3d_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r3d_kernel_stats.csv && head -8 gpurun_out/r3d_kernel_stats.csv
