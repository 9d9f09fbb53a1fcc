#!/bin/bash
# Round 2, run BT: final-tree rehearsal (encoder flash variants on pointer loads) --
# full GPU suite, smoke(), headline bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2bt_gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r2bt_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2bt_smoke.log 2>&1 || { tail -20 gpurun_out/r2bt_smoke.log; exit 1; }
tail -1 gpurun_out/r2bt_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r2bt_bench.json 2> gpurun_out/r2bt_bench.log || { tail -20 gpurun_out/r2bt_bench.log; exit 1; }
cut -c1-200 gpurun_out/r2bt_bench.json
exit $rc
