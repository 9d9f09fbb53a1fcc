#!/bin/bash
# Round 2, run BP: block-sparse flash kernels stage tiles through buffer resources -- sparse tests,
# sparse-vs-dense attention microbench, 20B BigBird seq 8k bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_sparse_flash.py tests/test_sparse_attention.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2bp_tests.log 2>&1 || { tail -40 gpurun_out/r2bp_tests.log; exit 1; }
tail -2 gpurun_out/r2bp_tests.log
timeout -k 10 300 python scripts/bench_sparse_attn.py > gpurun_out/r2bp_sparse_attn.jsonl 2> gpurun_out/r2bp_sparse_attn.log || { tail -20 gpurun_out/r2bp_sparse_attn.log; exit 1; }
cut -c1-250 gpurun_out/r2bp_sparse_attn.jsonl
timeout -k 10 500 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --steps 3 --warmup 2 > gpurun_out/r2bp_20b_bigbird_s8k.json 2> gpurun_out/r2bp_20b_bigbird_s8k.log || { tail -20 gpurun_out/r2bp_20b_bigbird_s8k.log; exit 1; }
cut -c1-200 gpurun_out/r2bp_20b_bigbird_s8k.json
