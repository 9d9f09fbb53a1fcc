#!/bin/bash
# Embedding backward keeps the weight shape from the forward: embedding / engine tests incl. the 2-rank ZeRO-3 path.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "embedding or multirank or overlapped or sharded or engine" > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3x_smoke.log 2>&1 || { tail -30 gpurun_out/r3x_smoke.log; exit 1; }
tail -1 gpurun_out/r3x_smoke.log
