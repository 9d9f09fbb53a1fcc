#!/bin/bash
# Round 2, run AI: selective-recompute stash parked in pinned host memory -- tests and A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_neox_stash_gpu.py tests/test_recompute_skip.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r2ai_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2ai_tests.log
[ $rc -le 1 ] || exit $rc
for o in 1 0; do
  DSA_STASH_OFFLOAD=$o timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2ai_o$o.json 2> gpurun_out/r2ai_o$o.log || { tail -20 gpurun_out/r2ai_o$o.log; exit 1; }
  echo "offload=$o $(grep -o 'selective recompute.*' gpurun_out/r2ai_o$o.log | tr '\n' ' ') $(grep -o 'stash safety.*' gpurun_out/r2ai_o$o.log) $(grep -o 'warmup 1.*' gpurun_out/r2ai_o$o.log | cut -c1-130) $(grep -o '"value": [0-9.]*' gpurun_out/r2ai_o$o.json) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r2ai_o$o.json)"
done
exit $rc
