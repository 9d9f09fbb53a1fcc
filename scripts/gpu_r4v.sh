#!/bin/bash
# Timed kernel profiles on the current tree: BERT-Large seq 128 b64, and the N=8-shaped GPT-NeoX-20B
# per-rank step on one GPU (--force-sharded --layers 6, micro-batch 8 x 2, no recompute).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4v_bert -o k --output-format csv -- python3 $R/scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 10 > $R/gpurun_out/r4v_bert.json 2> $R/gpurun_out/r4v_bert.log || { echo "bert rocprof failed"; tail -20 $R/gpurun_out/r4v_bert.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r4v_bert.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4v_n8 -o k --output-format csv -- python3 $R/bench.py --force-sharded --layers 6 --micro-batch 8 --grad-accum 2 --ckpt off --steps 3 --warmup 2 > $R/gpurun_out/r4v_n8.json 2> $R/gpurun_out/r4v_n8.log || { echo "n8 rocprof failed"; tail -20 $R/gpurun_out/r4v_n8.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r4v_n8.json
echo done
