#!/bin/bash
# Round 3: targeted GPU tests after the advisor fixes (fp32 split-K partials, overlap_step
# coverage) and a BERT-Large A/B point (split-K lives on the BERT shapes).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_fused_wgrad.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
for cfg in "128 64" "512 16"; do
  set -- $cfg
  timeout -k 10 300 python scripts/bench_bert.py --seq $1 --batch $2 > gpurun_out/r3b_bert_$1_$2.json 2> gpurun_out/r3b_bert_$1_$2.log || { tail -30 gpurun_out/r3b_bert_$1_$2.log; exit 1; }
  cat gpurun_out/r3b_bert_$1_$2.json
done
