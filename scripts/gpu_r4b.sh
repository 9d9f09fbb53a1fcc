#!/bin/bash
# D=128 dK/dV at one wave per SIMD (no scratch spill), fused ZeRO-2 cast-accumulate, ADVICE fixes:
# GPU tests of the changed paths, flash A/B, NeoX 1.3B ZeRO-2 and the 20B N=1 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lamb_overlap_gpu.py -x -q --timeout 200 --timeout-method thread -k "flash or embedding or lamb or sync_free or overlap" > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -1 gpurun_out/r4b_tests.log
timeout -k 10 200 python scripts/bench_attn.py --flash-only --D 96 128 64 > gpurun_out/r4b_attn_h64.jsonl 2> gpurun_out/r4b_attn.log || { tail -20 gpurun_out/r4b_attn.log; exit 1; }
cat gpurun_out/r4b_attn_h64.jsonl
DSA_FA_DKDV=31 timeout -k 10 200 python scripts/bench_attn.py --flash-only --D 96 > gpurun_out/r4b_attn_h64_occ1.jsonl 2>> gpurun_out/r4b_attn.log || { tail -20 gpurun_out/r4b_attn.log; exit 1; }
cat gpurun_out/r4b_attn_h64_occ1.jsonl
timeout -k 10 200 python scripts/bench_attn.py --flash-only --B 8 --H 16 --D 128 > gpurun_out/r4b_attn_13b.jsonl 2>> gpurun_out/r4b_attn.log || { tail -20 gpurun_out/r4b_attn.log; exit 1; }
cat gpurun_out/r4b_attn_13b.jsonl
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 --steps 20 --warmup 5 > gpurun_out/r4b_13b_mb8.json 2> gpurun_out/r4b_13b_mb8.log || { tail -30 gpurun_out/r4b_13b_mb8.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4b_13b_mb8.json
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 --micro-batch 16 --grad-accum 1 --steps 20 --warmup 5 > gpurun_out/r4b_13b_mb16.json 2> gpurun_out/r4b_13b_mb16.log || { tail -30 gpurun_out/r4b_13b_mb16.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4b_13b_mb16.json
timeout -k 10 420 python bench.py --steps 8 --warmup 3 > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.log || { tail -30 gpurun_out/r4b_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4b_bench.json
echo done
