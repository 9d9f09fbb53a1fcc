#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lamb" > gpurun_out/lamb_tests.log 2>&1 || { tail -40 gpurun_out/lamb_tests.log; exit 1; }
tail -2 gpurun_out/lamb_tests.log
for cfg in "128 64" "128 256" "512 16" "512 64"; do
  set -- $cfg
  timeout -k 10 300 python scripts/bench_bert.py --seq $1 --batch $2 > gpurun_out/bert_$1_$2.json 2> gpurun_out/bert_$1_$2.log || { tail -30 gpurun_out/bert_$1_$2.log; exit 1; }
  grep metric gpurun_out/bert_$1_$2.json
done
