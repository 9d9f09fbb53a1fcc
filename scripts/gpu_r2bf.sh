#!/bin/bash
# Round 2, run BF: shared transposed block-output gradient (parallel residual) -- GPU tests, then the
# 20B bench A/B on one box (default vs DSA_SHARE_GRAD_T=0).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gelu_transposed_gpu.py tests/test_neox_stash_gpu.py tests/test_kernels_gpu.py -k "gelu or wgrad or stash or rotary" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2bf_tests.log 2>&1 || { tail -40 gpurun_out/r2bf_tests.log; exit 1; }
tail -2 gpurun_out/r2bf_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r2bf_bench_new.json 2> gpurun_out/r2bf_bench_new.log || { tail -20 gpurun_out/r2bf_bench_new.log; exit 1; }
cut -c1-200 gpurun_out/r2bf_bench_new.json
DSA_SHARE_GRAD_T=0 timeout -k 10 400 python bench.py > gpurun_out/r2bf_bench_old.json 2> gpurun_out/r2bf_bench_old.log || { tail -20 gpurun_out/r2bf_bench_old.log; exit 1; }
cut -c1-200 gpurun_out/r2bf_bench_old.json
