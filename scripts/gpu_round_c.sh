#!/bin/bash
# flash-attention numerics + speed after the softmax/XCD changes, GEMM shape sweep,
# pipeline rehearsal (PP=2 over gloo on one GPU), then the flagship bench
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "flash or attention" > gpurun_out/flash_tests.log 2>&1 || { tail -30 gpurun_out/flash_tests.log; exit 1; }
tail -2 gpurun_out/flash_tests.log
timeout -k 10 300 python scripts/bench_attn.py > gpurun_out/attn.json 2> gpurun_out/attn.log || exit $?
cat gpurun_out/attn.json
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/gemm.json 2> gpurun_out/gemm.log || exit $?
cat gpurun_out/gemm.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --dist-backend gloo --model gpt-neox-125m --pipe 2 --optimizer onebitadam --freeze-step 2 --steps 2 --warmup 3 > gpurun_out/reh_pipe.json 2> gpurun_out/reh_pipe.log || { grep -A5 Error gpurun_out/reh_pipe.log | head -40; exit 1; }
cat gpurun_out/reh_pipe.json
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.log || exit $?
cat gpurun_out/bench_n1.json
grep warmup gpurun_out/bench_n1.log
