#!/bin/bash
# Multi-tensor sumsq: numerics, BERT-Large seq 128 A/B (HIP reduction vs torch _foreach_norm).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sumsq_multi_gpu.py tests/test_lamb_overlap_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4y_tests.log 2>&1 || { tail -40 gpurun_out/r4y_tests.log; exit 1; }
tail -1 gpurun_out/r4y_tests.log
bert() {  # tag seq batch env...
  tag=$1; seq=$2; b=$3; shift 3
  env "$@" timeout -k 10 300 python scripts/bench_bert.py --seq $seq --batch $b --steps 40 --warmup 10 > gpurun_out/r4y_bert_$tag.json 2> gpurun_out/r4y_bert_$tag.log || { tail -20 gpurun_out/r4y_bert_$tag.log; return 1; }
  echo "bert $tag $(grep -o '"value": [0-9.]*' gpurun_out/r4y_bert_$tag.json)"
}
bert multi 128 64 && bert foreach 128 64 DSA_SUMSQ_MULTI=0 && bert multi_b 128 64 && bert foreach_b 128 64 DSA_SUMSQ_MULTI=0 && bert multi512 512 16 && bert foreach512 512 16 DSA_SUMSQ_MULTI=0 || exit 1
echo done
