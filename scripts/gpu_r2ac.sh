#!/bin/bash
# Round 2, run AC: pipeline-parallel bench path (BASELINE config 4 shape: GPT-3 6.7B as a
# PipelineModule, 1F1B) rehearsed with PP ranks sharing one GPU over gloo (p2p staged via host).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for pp in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $pp --master-addr 127.0.0.1 \
    --master-port $((29800 + pp)) bench.py --gpus $pp --dist-backend gloo --model gpt3-6.7b --pipe $pp \
    --steps 2 --warmup 1 > gpurun_out/r2ac_pp$pp.json 2> gpurun_out/r2ac_pp$pp.log || { grep -v "^\s" gpurun_out/r2ac_pp$pp.log | tail -20; exit 1; }
  grep "\[bench\]" gpurun_out/r2ac_pp$pp.log | head -8
  tail -c 600 gpurun_out/r2ac_pp$pp.json
done
