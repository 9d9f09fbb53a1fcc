#!/bin/bash
# Round 2, run BO: flash fwd and dQ kernels also stage K / V tiles with buffer loads (fewer VGPRs;
# occupancy) -- attention tests, attention microbench A/B, 20B bench A/B (DSA_FA_BUFLOAD=1 vs 0), one box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_layer.py tests/test_sparse_flash.py tests/test_neox_stash_gpu.py -k "flash or attention or encoder or bert or stash or sparse" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2bo_tests.log 2>&1 || { tail -40 gpurun_out/r2bo_tests.log; exit 1; }
tail -2 gpurun_out/r2bo_tests.log
for rep in 1 2; do
  for b in 1 0; do
    DSA_FA_BUFLOAD=$b timeout -k 10 200 python scripts/bench_attn.py --flash-only --D 96 --iters 30 2>/dev/null | grep -v "^$" > gpurun_out/r2bo_attn_b$b.$rep.jsonl || exit 1
    echo "bufload=$b rep=$rep $(cat gpurun_out/r2bo_attn_b$b.$rep.jsonl | cut -c1-220)"
  done
done
for b in 1 0; do
  DSA_FA_BUFLOAD=$b timeout -k 10 400 python bench.py > gpurun_out/r2bo_bench_b$b.json 2> gpurun_out/r2bo_bench_b$b.log || { tail -20 gpurun_out/r2bo_bench_b$b.log; exit 1; }
  echo "bench bufload=$b $(cut -c60-110 gpurun_out/r2bo_bench_b$b.json)"
done
