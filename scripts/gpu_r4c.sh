#!/bin/bash
# Gathered 16-row blocks in the block-sparse flash kernels: GPU numerics tests, then the
# Fixed/16 (reference default block) and BigBird/64 benches against dense flash.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_sparse_flash.py tests/test_sparse_attention.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { tail -40 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode fixed --block 16 --seq 4096 --heads 16 --dim 64 --batch 4 --masked > gpurun_out/r4c_fixed16.jsonl 2> gpurun_out/r4c_bench.log || { tail -20 gpurun_out/r4c_bench.log; exit 1; }
cat gpurun_out/r4c_fixed16.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode fixed --block 32 --seq 4096 --heads 16 --dim 64 --batch 4 > gpurun_out/r4c_fixed32.jsonl 2>> gpurun_out/r4c_bench.log || { tail -20 gpurun_out/r4c_bench.log; exit 1; }
cat gpurun_out/r4c_fixed32.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode bigbird --block 16 --seq 4096 --heads 16 --dim 64 --batch 4 > gpurun_out/r4c_bigbird16.jsonl 2>> gpurun_out/r4c_bench.log || { tail -20 gpurun_out/r4c_bench.log; exit 1; }
cat gpurun_out/r4c_bigbird16.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode bigbird --block 64 --masked > gpurun_out/r4c_bigbird64.jsonl 2>> gpurun_out/r4c_bench.log || { tail -20 gpurun_out/r4c_bench.log; exit 1; }
cat gpurun_out/r4c_bigbird64.jsonl
echo done
