#!/bin/bash
# Rotary (padded vs unpadded LDS rows) and LayerNorm backward (row prefetch on / off) A/B, kernel tests.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "rotary or layernorm or layer_norm" --timeout 200 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1 || { tail -40 gpurun_out/r4g_tests.log; exit 1; }
tail -1 gpurun_out/r4g_tests.log
timeout -k 10 200 python scripts/bench_rotary.py --shape 4,2048,64,96,24 > gpurun_out/r4g_rotary.jsonl 2> gpurun_out/r4g_rotary.log || { tail -20 gpurun_out/r4g_rotary.log; exit 1; }
timeout -k 10 200 python scripts/bench_rotary.py --shape 16,2048,16,128,32 >> gpurun_out/r4g_rotary.jsonl 2>> gpurun_out/r4g_rotary.log || { tail -20 gpurun_out/r4g_rotary.log; exit 1; }
cat gpurun_out/r4g_rotary.jsonl
timeout -k 10 200 python scripts/bench_layernorm.py > gpurun_out/r4g_ln.jsonl 2> gpurun_out/r4g_ln.log || { tail -20 gpurun_out/r4g_ln.log; exit 1; }
cat gpurun_out/r4g_ln.jsonl
echo done
