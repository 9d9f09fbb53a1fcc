#!/bin/bash
# LDS-staged encoder key bias: encoder kernel tests, encoder attention micro-bench, BERT-Large (serial LAMB,
# 40 timed steps); then the 20B fill-source profile and the CU-masked Adam-overlap A/B (gpu_r3m.sh).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "encoder or qkv or transformer or flash" > gpurun_out/r3n_kernel_tests.log 2>&1 || { tail -40 gpurun_out/r3n_kernel_tests.log; exit 1; }
tail -1 gpurun_out/r3n_kernel_tests.log
timeout -k 10 200 python scripts/bench_encoder_attn.py > gpurun_out/r3n_encoder_attn.jsonl 2> gpurun_out/r3n_encoder_attn.log || { tail -30 gpurun_out/r3n_encoder_attn.log; exit 1; }
cat gpurun_out/r3n_encoder_attn.jsonl
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  timeout -k 10 200 python scripts/bench_bert.py --steps 40 --warmup 10 --seq $seq --batch $bs > gpurun_out/r3n_bert$seq.json 2> gpurun_out/r3n_bert$seq.log || { tail -30 gpurun_out/r3n_bert$seq.log; exit 1; }
  echo "bert $seq $(grep -o '"value": [0-9.]*' gpurun_out/r3n_bert$seq.json)"
done
bash scripts/gpu_r3m.sh
