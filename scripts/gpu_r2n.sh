#!/bin/bash
# Round 2, run N: split-K wgrad + autotuned forward GEMMs -- tests, BERT and 20B A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_lt_gpu.py tests/test_fused_wgrad.py tests/test_transformer_layer.py tests/test_engine_gpu.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r2n_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r2n_tests.log
[ $rc -le 1 ] || exit $rc
for cfg in "128 64" "512 16"; do
  set -- $cfg
  timeout -k 10 240 python scripts/bench_bert.py --seq $1 --batch $2 --steps 10 --warmup 3 2>/dev/null | grep '^{"metric' > gpurun_out/r2n_bert_s$1_b$2.json || exit 1
  cat gpurun_out/r2n_bert_s$1_b$2.json
done
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2n_bench.json 2> gpurun_out/r2n_bench.log || { tail -30 gpurun_out/r2n_bench.log; exit 1; }
tail -c 300 gpurun_out/r2n_bench.json
DSA_LINEAR_LT=0 timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2n_bench_nolt.json 2> gpurun_out/r2n_bench_nolt.log || { tail -30 gpurun_out/r2n_bench_nolt.log; exit 1; }
tail -c 300 gpurun_out/r2n_bench_nolt.json
exit $rc
