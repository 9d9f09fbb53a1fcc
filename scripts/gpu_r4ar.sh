#!/bin/bash
# r4ar: BERT encoder vs HF, seq 512 first (order / warmup check of r4aq)
set -o pipefail
mkdir -p gpurun_out/r4ar
cd /root/repo
timeout -k 10 600 python -u scripts/bench_bert_vs_hf.py --shapes 512x16,128x64 --iters 30 --warmup 10 > gpurun_out/r4ar/bert_vs_hf.jsonl 2> gpurun_out/r4ar/bert_vs_hf.err || { tail -20 gpurun_out/r4ar/bert_vs_hf.err; exit 1; }
cat gpurun_out/r4ar/bert_vs_hf.jsonl
