#!/bin/bash
# Round-4 starting point: timed kernel profiles of (1) the N=8-shaped per-rank 20B step on one GPU
# (--force-sharded, 6 layers, micro-batch 8 x 2, no recompute) and (2) BASELINE config 2 (NeoX 1.3B
# ZeRO-2), plus the 1.3B bench at micro-batch 8x2 and 16x1 over 20 timed steps.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4a_n8shape -o k --output-format csv -- python3 $R/bench.py --force-sharded --layers 6 --micro-batch 8 --grad-accum 2 --ckpt off --steps 3 --warmup 2 > $R/gpurun_out/r4a_n8shape.json 2> $R/gpurun_out/r4a_n8shape.log || { echo "n8shape rocprof failed"; tail -20 $R/gpurun_out/r4a_n8shape.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r4a_n8shape.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4a_13b -o k --output-format csv -- python3 $R/bench.py --model gpt-neox-1.3b --zero 2 --steps 5 --warmup 3 > $R/gpurun_out/r4a_13b_prof.json 2> $R/gpurun_out/r4a_13b_prof.log || { echo "1.3b rocprof failed"; tail -20 $R/gpurun_out/r4a_13b_prof.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r4a_13b_prof.json
cd $R
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 --steps 20 --warmup 5 > gpurun_out/r4a_13b_mb8.json 2> gpurun_out/r4a_13b_mb8.log || { tail -30 gpurun_out/r4a_13b_mb8.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4a_13b_mb8.json
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 --micro-batch 16 --grad-accum 1 --steps 20 --warmup 5 > gpurun_out/r4a_13b_mb16.json 2> gpurun_out/r4a_13b_mb16.log || { tail -30 gpurun_out/r4a_13b_mb16.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4a_13b_mb16.json
echo done
