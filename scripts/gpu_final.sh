#!/bin/bash
# End-of-session validation on a fresh box: GPU suite, smoke(), flagship N=1 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 420 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.log || { tail -30 gpurun_out/bench_final.log; exit 1; }
grep metric gpurun_out/bench_final.json
