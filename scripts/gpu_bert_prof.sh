#!/bin/bash
# rocprofv3 kernel stats of the BERT-Large seq-128 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log; exit 1; }
grep metric $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log
