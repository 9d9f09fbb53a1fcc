#!/bin/bash
# Round 2, run P: kernel profile of BERT-Large seq 512 / b16 (encoder flash, split-K wgrad).
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2p -o bert512 -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 512 --batch 16 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2p.log 2>&1 && echo profiled
