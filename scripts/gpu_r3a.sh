#!/bin/bash
# Round 3 first box: GPU suite, N=1 flagship bench, and the self-spawned 2-rank path
# (`bench.py --gpus 2`, no external launcher; gloo because two ranks share the one card).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3a_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3a_gpu_tests.log
timeout -k 10 420 python bench.py --steps 8 --warmup 4 > gpurun_out/r3a_bench_n1.json 2> gpurun_out/r3a_bench_n1.log || { tail -30 gpurun_out/r3a_bench_n1.log; exit 1; }
cat gpurun_out/r3a_bench_n1.json
DSA_MEMTRACE=1 timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --layers 6 --steps 1 --warmup 2 > gpurun_out/r3a_spawn_n2.json 2> gpurun_out/r3a_spawn_n2.log || { tail -30 gpurun_out/r3a_spawn_n2.log; exit 1; }
grep "\[bench\]" gpurun_out/r3a_spawn_n2.log | grep -v "mem after" 
cat gpurun_out/r3a_spawn_n2.json
