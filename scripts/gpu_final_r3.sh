#!/bin/bash
# End-of-round validation of the final tree: whole GPU suite, smoke(), the N=1 headline bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { tail -40 gpurun_out/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 420 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.log || { tail -30 gpurun_out/final_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/final_bench.json
bash scripts/gpu_r3w.sh
