#!/bin/bash
# Last check of the tree as committed (extension rebuilt by build()): GPU suite + smoke
export TMPDIR=/tmp
mkdir -p gpurun_out/final_c
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_c/gpu_tests.log 2>&1 || { tail -60 gpurun_out/final_c/gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_c/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_c/smoke.log 2>&1 || { tail -30 gpurun_out/final_c/smoke.log; exit 1; }
echo "smoke ok"
