#!/bin/bash
# Round 2, run G: kernel-level profile of block-sparse flash attention fwd+bwd (seq 8192 BigBird).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2g -o r2g -- python $GRAFT_REPO_ROOT/scripts/bench_sparse_attn.py --seq 8192 --heads 64 --dim 96 --mode bigbird --block 64 > $GRAFT_REPO_ROOT/gpurun_out/r2g.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r2g.log; exit 1; }
grep variant $GRAFT_REPO_ROOT/gpurun_out/r2g.log
