#!/bin/bash
# LN parameter-gradient accumulation into bound grads + cached zero placeholders: kernel / engine tests,
# 20B N=1 bench; RCCL probe with two ranks sharing the GPU.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_lamb_overlap_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1 || { tail -40 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
timeout -k 10 420 python bench.py --steps 6 --warmup 3 > gpurun_out/r3q_bench.json 2> gpurun_out/r3q_bench.log || { tail -30 gpurun_out/r3q_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3q_bench.json
timeout -k 10 200 python scripts/rccl_two_ranks_one_gpu.py > gpurun_out/r3q_rccl_probe.jsonl 2> gpurun_out/r3q_rccl_probe.log; echo "rccl probe rc=$?"
cat gpurun_out/r3q_rccl_probe.jsonl; tail -5 gpurun_out/r3q_rccl_probe.log
