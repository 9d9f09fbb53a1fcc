#!/bin/bash
# Round 2, run BG: regression records of the other BASELINE configs on the current tree
# (GPT-NeoX 1.3B ZeRO-2 with the dual-output GeLU backward, BERT-Large seq 128 / 512, 20B BigBird seq 8k).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 > gpurun_out/r2bg_neox1.3b_zero2.json 2> gpurun_out/r2bg_neox1.3b_zero2.log || { tail -20 gpurun_out/r2bg_neox1.3b_zero2.log; exit 1; }
cut -c1-220 gpurun_out/r2bg_neox1.3b_zero2.json
timeout -k 10 240 python scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2bg_bert_seq128_b64.json || exit 1
cut -c1-220 gpurun_out/r2bg_bert_seq128_b64.json
timeout -k 10 240 python scripts/bench_bert.py --seq 512 --batch 16 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2bg_bert_seq512_b16.json || exit 1
cut -c1-220 gpurun_out/r2bg_bert_seq512_b16.json
timeout -k 10 500 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --steps 3 --warmup 2 > gpurun_out/r2bg_20b_bigbird_s8k.json 2> gpurun_out/r2bg_20b_bigbird_s8k.log || { tail -20 gpurun_out/r2bg_20b_bigbird_s8k.log; exit 1; }
cut -c1-220 gpurun_out/r2bg_20b_bigbird_s8k.json
