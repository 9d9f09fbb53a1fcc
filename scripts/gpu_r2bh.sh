#!/bin/bash
# Round 2, run BH: final-tree rehearsal -- full GPU suite, smoke(), headline bench, kernel profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2bh_gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r2bh_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2bh_smoke.log 2>&1 || { tail -20 gpurun_out/r2bh_smoke.log; exit 1; }
tail -1 gpurun_out/r2bh_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r2bh_bench.json 2> gpurun_out/r2bh_bench.log || { tail -20 gpurun_out/r2bh_bench.log; exit 1; }
cut -c1-200 gpurun_out/r2bh_bench.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2bh -o neox -- python $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r2bh_prof_bench.json 2> $R/gpurun_out/r2bh_prof_bench.log || { tail -20 $R/gpurun_out/r2bh_prof_bench.log; exit 1; }
echo profiled
exit $rc
