#!/bin/bash
# r4at: timed kernel profile of the N=8-shaped GPT-NeoX-20B per-rank step on the final round-4 tree
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r4at_n8 -o k --output-format csv -- python3 $R/bench.py --force-sharded --layers 6 --micro-batch 8 --grad-accum 2 --ckpt off --steps 3 --warmup 2 > $R/gpurun_out/r4at_n8.json 2> $R/gpurun_out/r4at_n8.log || { echo "n8 rocprof failed"; tail -20 $R/gpurun_out/r4at_n8.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r4at_n8.json
