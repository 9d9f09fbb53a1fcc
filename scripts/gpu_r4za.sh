#!/bin/bash
# D = 128 flash tiles with a 304-byte LDS row stride: numerics, bank-conflict counters, kernel times,
# GPT-NeoX 1.3B ZeRO-2 step.
export TMPDIR=/tmp
mkdir -p gpurun_out/r4za_pmc
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_sparse_flash.py tests/test_neox_stash_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4za_tests.log 2>&1 || { tail -40 gpurun_out/r4za_tests.log; exit 1; }
tail -1 gpurun_out/r4za_tests.log
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d $R/gpurun_out/r4za_pmc/d128 -o run --output-format csv -- python $R/scripts/bench_attn.py --D 128 --iters 3 --flash-only > $R/gpurun_out/r4za_pmc/d128.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/r4za_pmc/d128.log; exit 1; }
cd $R
timeout -k 10 300 python scripts/bench_attn.py --D 128 96 --flash-only > gpurun_out/r4za_attn.jsonl 2> gpurun_out/r4za_attn.log || { tail -20 gpurun_out/r4za_attn.log; exit 1; }
cat gpurun_out/r4za_attn.jsonl
timeout -k 10 300 python scripts/bench_attn.py --B 8 --H 16 --D 128 --flash-only > gpurun_out/r4za_attn13b.jsonl 2>> gpurun_out/r4za_attn.log || exit 1
cat gpurun_out/r4za_attn13b.jsonl
timeout -k 10 400 python bench.py --model gpt-neox-1.3b --zero 2 --steps 20 --warmup 5 > gpurun_out/r4za_13b.json 2> gpurun_out/r4za_13b.log || { tail -20 gpurun_out/r4za_13b.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4za_13b.json
echo done
