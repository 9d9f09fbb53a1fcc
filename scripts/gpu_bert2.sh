#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "softmax or transformer or attention_matches" > gpurun_out/sm_tests.log 2>&1 || { tail -40 gpurun_out/sm_tests.log; exit 1; }
tail -2 gpurun_out/sm_tests.log
for cfg in "128 64" "512 16"; do
  set -- $cfg
  timeout -k 10 300 python scripts/bench_bert.py --seq $1 --batch $2 > gpurun_out/bert_$1_$2.json 2> gpurun_out/bert_$1_$2.log || { tail -30 gpurun_out/bert_$1_$2.log; exit 1; }
  grep metric gpurun_out/bert_$1_$2.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log; exit 1; }
