#!/bin/bash
# BERT-Large seq-512 regression hunt: same-box A/B of the split-K weight gradient, and a kernel profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
B="python scripts/bench_bert.py --steps 10 --warmup 3 --overlap-step off"
timeout -k 10 200 $B --seq 512 --batch 16 > gpurun_out/r3k_512_base.json 2> gpurun_out/r3k_512_base.log || { tail -30 gpurun_out/r3k_512_base.log; exit 1; }
grep metric gpurun_out/r3k_512_base.json
DSA_WGRAD_SPLIT=1 timeout -k 10 200 $B --seq 512 --batch 16 > gpurun_out/r3k_512_nosplit.json 2> gpurun_out/r3k_512_nosplit.log || { tail -30 gpurun_out/r3k_512_nosplit.log; exit 1; }
grep metric gpurun_out/r3k_512_nosplit.json
timeout -k 10 200 $B --seq 128 --batch 64 > gpurun_out/r3k_128_base.json 2> gpurun_out/r3k_128_base.log || { tail -30 gpurun_out/r3k_128_base.log; exit 1; }
grep metric gpurun_out/r3k_128_base.json
DSA_WGRAD_SPLIT=1 timeout -k 10 200 $B --seq 128 --batch 64 > gpurun_out/r3k_128_nosplit.json 2> gpurun_out/r3k_128_nosplit.log || { tail -30 gpurun_out/r3k_128_nosplit.log; exit 1; }
grep metric gpurun_out/r3k_128_nosplit.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3k_prof_bert512 -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 512 --batch 16 --steps 5 --warmup 2 --overlap-step off > $GRAFT_REPO_ROOT/gpurun_out/r3k_prof_bert512.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3k_prof_bert512.log; exit 1; }
echo profiled
