#!/bin/bash
# Overlapped LAMB step: exactness tests, then BERT-Large with the step overlapped vs serial.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_lamb_overlap_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3j_lamb_overlap_tests.log 2>&1 || { tail -40 gpurun_out/r3j_lamb_overlap_tests.log; exit 1; }
tail -2 gpurun_out/r3j_lamb_overlap_tests.log
for ov in on off; do
timeout -k 10 200 python scripts/bench_bert.py --seq 128 --batch 64 --steps 10 --warmup 3 --overlap-step $ov > gpurun_out/r3j_bert128_$ov.json 2> gpurun_out/r3j_bert128_$ov.log || { tail -30 gpurun_out/r3j_bert128_$ov.log; exit 1; }
cat gpurun_out/r3j_bert128_$ov.json
timeout -k 10 200 python scripts/bench_bert.py --seq 512 --batch 16 --steps 10 --warmup 3 --overlap-step $ov > gpurun_out/r3j_bert512_$ov.json 2> gpurun_out/r3j_bert512_$ov.log || { tail -30 gpurun_out/r3j_bert512_$ov.log; exit 1; }
cat gpurun_out/r3j_bert512_$ov.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3j_prof_bert -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3j_prof_bert.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3j_prof_bert.log; exit 1; }
echo bert profiled
