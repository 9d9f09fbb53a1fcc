#!/bin/bash
# Round 2, run AG: overlapped optimizer step (bound ZeRO-3) -- exactness tests and same-box A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2ag_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2ag_tests.log
[ $rc -le 1 ] || exit $rc
for o in 1 0 1; do
  DSA_OVERLAP_STEP=$o timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2ag_o$o.json 2> gpurun_out/r2ag_o$o.log || { tail -20 gpurun_out/r2ag_o$o.log; exit 1; }
  echo "overlap=$o $(grep -o 'warmup 1.*' gpurun_out/r2ag_o$o.log | cut -c1-120) $(grep -o '"value": [0-9.]*' gpurun_out/r2ag_o$o.json) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r2ag_o$o.json)"
done
exit $rc
