#!/bin/bash
# Gain-gated measured hipBLASLt routes (DSA_LT=1): numerics, then A/B on BERT-Large seq 128 / 512,
# GPT-NeoX 1.3B ZeRO-2 and the 20B N=1 step.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_lt_tune_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4u_tests.log 2>&1 || { tail -40 gpurun_out/r4u_tests.log; exit 1; }
tail -1 gpurun_out/r4u_tests.log
bert() {  # tag seq batch env...
  tag=$1; seq=$2; b=$3; shift 3
  env "$@" timeout -k 10 300 python scripts/bench_bert.py --seq $seq --batch $b --steps 40 --warmup 10 > gpurun_out/r4u_bert_$tag.json 2> gpurun_out/r4u_bert_$tag.log || { tail -20 gpurun_out/r4u_bert_$tag.log; return 1; }
  echo "bert $tag $(grep -o '"value": [0-9.]*' gpurun_out/r4u_bert_$tag.json)"
}
neox() {  # tag env... (args after --)
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py $NEOX_ARGS > gpurun_out/r4u_$tag.json 2> gpurun_out/r4u_$tag.log || { tail -20 gpurun_out/r4u_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4u_$tag.json)"
}
bert lt128 128 64 DSA_LT=1 && bert base128 128 64 DSA_LT=0 && bert lt128b 128 64 DSA_LT=1 && bert base128b 128 64 DSA_LT=0 || exit 1
bert lt512 512 16 DSA_LT=1 && bert base512 512 16 DSA_LT=0 || exit 1
NEOX_ARGS="--model gpt-neox-1.3b --zero 2 --steps 20 --warmup 5"
neox lt13b DSA_LT=1 && neox base13b DSA_LT=0 && neox lt13b_b DSA_LT=1 || exit 1
NEOX_ARGS="--steps 6 --warmup 3"
neox lt20b DSA_LT=1 && neox base20b DSA_LT=0 || exit 1
echo done
