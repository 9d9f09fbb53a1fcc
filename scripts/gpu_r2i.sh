#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gemm_lt_gpu.py -x -v --timeout 100 --timeout-method thread > gpurun_out/r2i_tests.log 2>&1 || { tail -40 gpurun_out/r2i_tests.log; exit 1; }
tail -2 gpurun_out/r2i_tests.log
timeout -k 10 200 python scripts/bench_gemm_epilogue.py --tokens 8192 > gpurun_out/r2i_gemm_epi.jsonl 2> gpurun_out/r2i_gemm_epi.log || { tail -20 gpurun_out/r2i_gemm_epi.log; exit 1; }
cat gpurun_out/r2i_gemm_epi.jsonl
