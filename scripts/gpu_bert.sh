#!/bin/bash
# BERT-Large pre-training throughput on one MI355X.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for cfg in "128 64" "128 256" "512 16" "512 64"; do
  set -- $cfg
  timeout -k 10 300 python scripts/bench_bert.py --seq $1 --batch $2 > gpurun_out/bert_$1_$2.json 2> gpurun_out/bert_$1_$2.log || { tail -30 gpurun_out/bert_$1_$2.log; exit 1; }
  cat gpurun_out/bert_$1_$2.json
done
