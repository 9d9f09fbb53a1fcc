#!/bin/bash
# Round 2, run V: merged dK/dV + dQ flash backward launch -- tests, BERT and 20B A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_layer.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r2v_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r2v_tests.log
[ $rc -le 1 ] || exit $rc
for m in 1 0; do
  for cfg in "128 64" "512 16"; do
    set -- $cfg
    DSA_FLASH_BWD_MERGE=$m timeout -k 10 240 python scripts/bench_bert.py --seq $1 --batch $2 --steps 10 --warmup 3 2>/dev/null | grep '^{"metric' > gpurun_out/r2v_bert_s$1_b$2_m$m.json || exit 1
    echo "merge=$m $(cut -c1-120 gpurun_out/r2v_bert_s$1_b$2_m$m.json)"
  done
done
for m in 1 0; do
  DSA_FLASH_BWD_MERGE=$m timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2v_bench_m$m.json 2> gpurun_out/r2v_bench_m$m.log || { tail -20 gpurun_out/r2v_bench_m$m.log; exit 1; }
  echo "merge=$m $(tail -c 700 gpurun_out/r2v_bench_m$m.json | head -c 200)"
done
exit $rc
