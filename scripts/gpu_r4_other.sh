#!/bin/bash
# Other BASELINE configs on the final round-4 tree: 20B ZeRO-3 at seq 8192 with BigBird block-sparse and
# with dense causal flash attention.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --steps 6 --warmup 3 > gpurun_out/r4_bigbird_s8k.json 2> gpurun_out/r4_bigbird_s8k.log || { tail -30 gpurun_out/r4_bigbird_s8k.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_bigbird_s8k.json


echo done
