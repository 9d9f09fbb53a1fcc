#!/bin/bash
# Offload configs on the final round-4 tree: GPT-3 6.7B ZeRO-Offload (optimizer on the CPU, pipelined) and
# ZeRO-Infinity 5.2B NeoX with optimizer states on NVMe, BigBird seq 8192.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python bench.py --model gpt3-6.7b --offload all --ckpt on --steps 4 --warmup 2 > gpurun_out/r4ae_67b_offload.json 2> gpurun_out/r4ae_67b_offload.log || { tail -30 gpurun_out/r4ae_67b_offload.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4ae_67b_offload.json
timeout -k 10 700 python bench.py --hidden 4096 --layers 24 --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --offload nvme --steps 3 --warmup 1 > gpurun_out/r4ae_5b_nvme.json 2> gpurun_out/r4ae_5b_nvme.log || { tail -30 gpurun_out/r4ae_5b_nvme.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4ae_5b_nvme.json
echo done
