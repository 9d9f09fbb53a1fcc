#!/bin/bash
# BERT head-layout kernels: numerics test, BERT-Large bench, rocprof kernel stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_layer.py tests/test_bert_model.py -x -v --timeout 120 --timeout-method thread -k "head or postln or preln or dropout or bert" > gpurun_out/heads_tests.log 2>&1 || { tail -40 gpurun_out/heads_tests.log; exit 1; }
tail -3 gpurun_out/heads_tests.log
for cfg in "128 64" "512 16"; do
  set -- $cfg
  timeout -k 10 300 python scripts/bench_bert.py --seq $1 --batch $2 > gpurun_out/bertH_$1_$2.json 2> gpurun_out/bertH_$1_$2.log || { tail -30 gpurun_out/bertH_$1_$2.log; exit 1; }
  cat gpurun_out/bertH_$1_$2.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bertH -o run --output-format csv -- python $R/scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 2 > $R/gpurun_out/prof_bertH.log 2>&1 || { tail -30 $R/gpurun_out/prof_bertH.log; exit 1; }
grep metric $R/gpurun_out/prof_bertH.log
