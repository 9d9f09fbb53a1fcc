#!/bin/bash
# Round 2, run F: block-sparse flash attention numerics + the seq-8192 attention benchmark
# (single-stage LDS default vs register-prefetch variant).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sparse_flash.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1 || { tail -40 gpurun_out/r2f_tests.log; exit 1; }
tail -3 gpurun_out/r2f_tests.log
timeout -k 10 300 python scripts/bench_sparse_attn.py --seq 8192 --heads 64 --dim 96 --mode bigbird --block 64 --unfused > gpurun_out/r2f_attn_bench.jsonl 2> gpurun_out/r2f_attn_bench.log || { tail -20 gpurun_out/r2f_attn_bench.log; exit 1; }
DSA_SPARSE_FLASH_RP=1 timeout -k 10 300 python scripts/bench_sparse_attn.py --seq 8192 --heads 64 --dim 96 --mode bigbird --block 64 >> gpurun_out/r2f_attn_bench.jsonl 2>> gpurun_out/r2f_attn_bench.log || { tail -20 gpurun_out/r2f_attn_bench.log; exit 1; }
cat gpurun_out/r2f_attn_bench.jsonl
