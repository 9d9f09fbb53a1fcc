#!/bin/bash
# r4aq: BERT-Large encoder fwd+bwd, DeepSpeedTransformerLayer stack vs HuggingFace BertModel (sdpa / eager)
set -o pipefail
mkdir -p gpurun_out/r4aq
cd /root/repo
timeout -k 10 600 python -u scripts/bench_bert_vs_hf.py --shapes 384x32,128x64,512x16 --iters 20 > gpurun_out/r4aq/bert_vs_hf.jsonl 2> gpurun_out/r4aq/bert_vs_hf.err || { tail -20 gpurun_out/r4aq/bert_vs_hf.err; exit 1; }
cat gpurun_out/r4aq/bert_vs_hf.jsonl
