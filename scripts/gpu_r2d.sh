#!/bin/bash
# Round 2, run D: GPU suite on the current tree, headline bench (bypass), N=2 memory-plan rehearsal
# (2 gloo ranks sharing the card, 22 of 44 layers each, sharded ZeRO-3 path with prefetch window + pool).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2d_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r2d_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2d_gpu_tests.log
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2d_bench.json 2> gpurun_out/r2d_bench.log || { tail -30 gpurun_out/r2d_bench.log; exit 1; }
tail -c 600 gpurun_out/r2d_bench.json
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29702 bench.py --gpus 2 --dist-backend gloo --layers 22 --steps 1 --warmup 1 \
    > gpurun_out/r2d_reh_n2.json 2> gpurun_out/r2d_reh_n2.log || { grep -v "^\[rank1\]" gpurun_out/r2d_reh_n2.log | tail -30; exit 1; }
grep "\[bench\]" gpurun_out/r2d_reh_n2.log
tail -c 700 gpurun_out/r2d_reh_n2.json
