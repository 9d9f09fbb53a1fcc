#!/bin/bash
# Round 2, run BL: in-place cross-entropy backward -- GPU tests, then the 20B bench A/B on one box
# (default vs DSA_XENT_INPLACE=0: memory peak, stashed layers, tokens/s).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "cross_entropy or neox or zero3" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2bl_tests.log 2>&1 || { tail -40 gpurun_out/r2bl_tests.log; exit 1; }
tail -2 gpurun_out/r2bl_tests.log
for v in 1 0; do
  DSA_XENT_INPLACE=$v timeout -k 10 400 python bench.py > gpurun_out/r2bl_x$v.json 2> gpurun_out/r2bl_x$v.log || { tail -20 gpurun_out/r2bl_x$v.log; exit 1; }
  echo "inplace=$v $(cut -c60-125 gpurun_out/r2bl_x$v.json) $(grep -o 'selective recompute: [0-9]*/44.*' gpurun_out/r2bl_x$v.log) $(grep 'warmup 0' gpurun_out/r2bl_x$v.log | grep -o 'peak=.*')"
done
