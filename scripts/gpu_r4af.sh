#!/bin/bash
# Peak parameters on one GPU on the final round-4 tree: 30.3B NeoX-style model, Adam moments in pinned host memory.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python bench.py --hidden 7168 --layers 48 --offload moments --steps 3 --warmup 2 > gpurun_out/r4af_30b.json 2> gpurun_out/r4af_30b.log || { tail -30 gpurun_out/r4af_30b.log; exit 1; }
grep -o '"value": [0-9.]*\|"params_per_gpu": [0-9.]*\|"stashed_attention_layers": [0-9]*\|"peak_hbm_gib": [0-9.]*' gpurun_out/r4af_30b.json
echo done
