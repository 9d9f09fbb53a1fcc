#!/bin/bash
# Round 2, run AB: LayerNorm residual passthrough in the GPT-NeoX block -- GPU tests + 20B profile + bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_recompute_skip.py tests/test_kernels_gpu.py tests/test_zero3_pool.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2ab_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2ab_tests.log
[ $rc -le 1 ] || exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2ab -o neox -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2ab_prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2ab_prof_bench.log && echo profiled
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2ab_bench.json 2> gpurun_out/r2ab_bench.log || { tail -20 gpurun_out/r2ab_bench.log; exit 1; }
tail -c 700 gpurun_out/r2ab_bench.json | head -c 200
exit $rc
