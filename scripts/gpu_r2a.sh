#!/bin/bash
# Round 2, run A: GPU suite (incl. the RCCL world-1 sharded ZeRO-3 parity tests), then the
# 20B headline bench on the bypass path and on the forced sharded path.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r2a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r2a_gpu_tests.log
timeout -k 10 420 python bench.py --steps 4 --warmup 2 > gpurun_out/r2a_bench.json 2> gpurun_out/r2a_bench.log || { tail -30 gpurun_out/r2a_bench.log; exit 1; }
cat gpurun_out/r2a_bench.json
timeout -k 10 420 python bench.py --steps 4 --warmup 2 --force-sharded > gpurun_out/r2a_bench_sharded.json 2> gpurun_out/r2a_bench_sharded.log || { tail -30 gpurun_out/r2a_bench_sharded.log; exit 1; }
cat gpurun_out/r2a_bench_sharded.json
