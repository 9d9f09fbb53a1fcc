#!/bin/bash
# Round 2, run L: encoder flash attention (key bias + in-kernel dropout) tests, BERT A/B, profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_layer.py -m gpu -q -k "encoder or memory_modes or flash" --timeout 120 --timeout-method thread > gpurun_out/r2l_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r2l_tests.log
[ $rc -le 1 ] || exit $rc
for cfg in "128 64" "512 16" "128 256" "512 64"; do
  set -- $cfg
  timeout -k 10 240 python scripts/bench_bert.py --seq $1 --batch $2 --steps 10 --warmup 3 > gpurun_out/r2l_bert_s$1_b$2.json 2> gpurun_out/r2l_bert_s$1_b$2.log || { tail -20 gpurun_out/r2l_bert_s$1_b$2.log; exit 1; }
  cat gpurun_out/r2l_bert_s$1_b$2.json
done
DSA_ENCODER_FLASH=0 timeout -k 10 240 python scripts/bench_bert.py --seq 128 --batch 64 --steps 10 --warmup 3 > gpurun_out/r2l_bert_s128_b64_noflash.json 2>/dev/null && cat gpurun_out/r2l_bert_s128_b64_noflash.json
DSA_ENCODER_FLASH=0 timeout -k 10 240 python scripts/bench_bert.py --seq 512 --batch 16 --steps 10 --warmup 3 > gpurun_out/r2l_bert_s512_b16_noflash.json 2>/dev/null && cat gpurun_out/r2l_bert_s512_b16_noflash.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2l -o bert -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 2 > /dev/null 2>&1 && echo profiled
exit $rc
