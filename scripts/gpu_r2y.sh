#!/bin/bash
# Round 2, run Y: kernel profile of the headline GPT-NeoX-20B step (bound path).
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2y -o neox -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2y_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2y_bench.log && echo profiled
