#!/bin/bash
# Round 2, run W: fused short-sequence flash backward -- tests + BERT + profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_layer.py tests/test_fused_wgrad.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r2w_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r2w_tests.log
[ $rc -le 1 ] || exit $rc
for cfg in "128 64" "512 16"; do
  set -- $cfg
  timeout -k 10 240 python scripts/bench_bert.py --seq $1 --batch $2 --steps 10 --warmup 3 2>/dev/null | grep '^{"metric' > gpurun_out/r2w_bert_s$1_b$2.json || exit 1
  cat gpurun_out/r2w_bert_s$1_b$2.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2w -o bert -- python $GRAFT_REPO_ROOT/scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 2 > /dev/null 2>&1 && echo profiled
exit $rc
