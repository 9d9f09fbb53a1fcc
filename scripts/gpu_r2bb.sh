#!/bin/bash
# Round 2, run BB: transposing bias+GeLU kernels -- numerics tests, NeoX recompute equivalence,
# then a same-box A/B of the 20B bench (new default vs DSA_COLMAJOR_GELU=0 DSA_DUAL_GELU_BWD=0).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gelu_transposed_gpu.py tests/test_neox_stash_gpu.py tests/test_kernels_gpu.py -k "gelu or transpose or wgrad or stash" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2bb_tests.log 2>&1 || { tail -40 gpurun_out/r2bb_tests.log; exit 1; }
tail -2 gpurun_out/r2bb_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r2bb_bench_new.json 2> gpurun_out/r2bb_bench_new.log || { tail -20 gpurun_out/r2bb_bench_new.log; exit 1; }
cut -c1-200 gpurun_out/r2bb_bench_new.json
DSA_COLMAJOR_GELU=0 DSA_DUAL_GELU_BWD=0 timeout -k 10 400 python bench.py > gpurun_out/r2bb_bench_old.json 2> gpurun_out/r2bb_bench_old.log || { tail -20 gpurun_out/r2bb_bench_old.log; exit 1; }
cut -c1-200 gpurun_out/r2bb_bench_old.json
