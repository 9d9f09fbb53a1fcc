#!/bin/bash
# bench N=1 flagship, memory-planner calibration, and 2-rank rehearsals on one GPU (gloo)
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.log || exit $?
cat gpurun_out/bench_n1.json
timeout -k 10 300 python bench.py --layers 8 --ckpt off --offload none --steps 2 --warmup 1 --max-live 0 > gpurun_out/cal_l8.json 2> gpurun_out/cal_l8.log || exit $?
cat gpurun_out/cal_l8.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dist-backend gloo --model gpt-neox-1.3b --steps 2 --warmup 1 > gpurun_out/reh_z3.json 2> gpurun_out/reh_z3.log || exit $?
cat gpurun_out/reh_z3.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --dist-backend gloo --model gpt-neox-125m --pipe 2 --optimizer onebitadam --freeze-step 2 --steps 2 --warmup 3 > gpurun_out/reh_pipe.json 2> gpurun_out/reh_pipe.log || exit $?
cat gpurun_out/reh_pipe.json
