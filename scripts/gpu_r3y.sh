#!/bin/bash
# Other BASELINE configs on the final round-3 tree: GPT-NeoX 1.3B ZeRO-2 and 20B ZeRO-3 BigBird seq 8192.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python bench.py --model gpt-neox-1.3b --zero 2 > gpurun_out/r3y_neox13b_zero2.json 2> gpurun_out/r3y_neox13b_zero2.log || { tail -30 gpurun_out/r3y_neox13b_zero2.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3y_neox13b_zero2.json
timeout -k 10 600 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird > gpurun_out/r3y_20b_bigbird_s8k.json 2> gpurun_out/r3y_20b_bigbird_s8k.log || { tail -30 gpurun_out/r3y_20b_bigbird_s8k.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3y_20b_bigbird_s8k.json
