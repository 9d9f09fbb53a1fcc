#!/bin/bash
# Final round-4 tree (after PLD / HF sparse attention changes): full GPU test suite, smoke(), the
# default bench (driver contract)
export TMPDIR=/tmp
mkdir -p gpurun_out/final_b
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_b/gpu_tests.log 2>&1 || { tail -60 gpurun_out/final_b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_b/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_b/smoke.log 2>&1 || { tail -30 gpurun_out/final_b/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/final_b/bench.json 2> gpurun_out/final_b/bench.log || { tail -30 gpurun_out/final_b/bench.log; exit 1; }
cut -c1-400 gpurun_out/final_b/bench.json
