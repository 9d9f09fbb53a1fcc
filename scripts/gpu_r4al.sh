#!/bin/bash
# r4al: BERT-Large progressive layer drop (BASELINE row 20) and batch-1 max sequence, dense vs
# block-sparse (row 15)
set -o pipefail
mkdir -p gpurun_out/r4al
cd /root/repo
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sparse_flash.py -k "masked_fused or hf" > gpurun_out/r4al/tests.log 2>&1 || exit 1
for pld in 0 0.5; do
  timeout -k 10 300 python -u scripts/bench_bert.py --seq 128 --batch 64 --steps 40 --warmup 10 --pld $pld > gpurun_out/r4al/bert128_pld$pld.json 2> gpurun_out/r4al/bert128_pld$pld.err || exit 1
done
for pld in 0 0.5; do
  timeout -k 10 300 python -u scripts/bench_bert.py --seq 512 --batch 16 --steps 40 --warmup 10 --pld $pld > gpurun_out/r4al/bert512_pld$pld.json 2> gpurun_out/r4al/bert512_pld$pld.err || exit 1
done
timeout -k 10 900 python -u scripts/bench_sparse_maxseq.py --model bert-large > gpurun_out/r4al/maxseq_large.jsonl 2> gpurun_out/r4al/maxseq_large.err || exit 1
