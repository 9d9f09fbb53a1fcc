#!/bin/bash
# r4am: batch-1 max sequence, BERT-Large: HF dense eager vs HF + block-sparse vs this framework's flash encoder
set -o pipefail
mkdir -p gpurun_out/r4am
cd /root/repo
timeout -k 10 1000 python -u scripts/bench_sparse_maxseq.py --model bert-large > gpurun_out/r4am/maxseq_large.jsonl 2> gpurun_out/r4am/maxseq_large.err || exit 1
