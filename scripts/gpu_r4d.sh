#!/bin/bash
# Gathered-block sparse flash (tests + benches) and the side-stream weight-transpose prefetch
# (exactness test + same-box 20B A/B).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_sparse_flash.py tests/test_sparse_attention.py tests/test_wt_prefetch_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1 || { tail -40 gpurun_out/r4d_tests.log; exit 1; }
tail -1 gpurun_out/r4d_tests.log
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode fixed --block 16 --seq 4096 --heads 16 --dim 64 --batch 4 --masked > gpurun_out/r4d_fixed16.jsonl 2> gpurun_out/r4d_bench.log || { tail -20 gpurun_out/r4d_bench.log; exit 1; }
cat gpurun_out/r4d_fixed16.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode fixed --block 32 --seq 4096 --heads 16 --dim 64 --batch 4 > gpurun_out/r4d_fixed32.jsonl 2>> gpurun_out/r4d_bench.log || { tail -20 gpurun_out/r4d_bench.log; exit 1; }
cat gpurun_out/r4d_fixed32.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode bigbird --block 16 --seq 4096 --heads 16 --dim 64 --batch 4 > gpurun_out/r4d_bigbird16.jsonl 2>> gpurun_out/r4d_bench.log || { tail -20 gpurun_out/r4d_bench.log; exit 1; }
cat gpurun_out/r4d_bigbird16.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode bigbird --block 64 --masked > gpurun_out/r4d_bigbird64.jsonl 2>> gpurun_out/r4d_bench.log || { tail -20 gpurun_out/r4d_bench.log; exit 1; }
cat gpurun_out/r4d_bigbird64.jsonl
for pf in 0 1; do
  DSA_WT_PREFETCH=$pf timeout -k 10 420 python bench.py --steps 6 --warmup 3 > gpurun_out/r4d_bench_pf$pf.json 2> gpurun_out/r4d_bench_pf$pf.log || { tail -30 gpurun_out/r4d_bench_pf$pf.log; exit 1; }
  echo "prefetch=$pf $(grep -o '"value": [0-9.]*' gpurun_out/r4d_bench_pf$pf.json)"
done
echo done
