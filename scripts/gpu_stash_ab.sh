#!/bin/bash
# Selective-recompute (attention stash) test + 20B bench A/B on one box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_neox_stash_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stash or colsum or layernorm or bias_gelu or transpose" > gpurun_out/stash_tests.log 2>&1 || { tail -40 gpurun_out/stash_tests.log; exit 1; }
tail -2 gpurun_out/stash_tests.log
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_st1.json 2> gpurun_out/bench_st1.log || { tail -30 gpurun_out/bench_st1.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_st1.log
cat gpurun_out/bench_st1.json
timeout -k 10 400 env DSA_STASH=0 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_st0.json 2> gpurun_out/bench_st0.log || { tail -30 gpurun_out/bench_st0.log; exit 1; }
cat gpurun_out/bench_st0.json
