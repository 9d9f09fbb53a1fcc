#!/bin/bash
# Transposed-operand wgrad: kernel tests, GEMM formulation sweep, full 20B bench A/B on one box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "transpose or wgrad_transposed or colsum or extension" > gpurun_out/nt_tests.log 2>&1 || { tail -40 gpurun_out/nt_tests.log; exit 1; }
tail -2 gpurun_out/nt_tests.log
true
true
timeout -k 10 400 env DSA_DGRAD_NT=1 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_dg1.json 2> gpurun_out/bench_dg1.log || { tail -30 gpurun_out/bench_dg1.log; exit 1; }
cat gpurun_out/bench_dg1.json
timeout -k 10 400 env DSA_DGRAD_NT=0 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_dg0.json 2> gpurun_out/bench_dg0.log || { tail -30 gpurun_out/bench_dg0.log; exit 1; }
cat gpurun_out/bench_dg0.json
