#!/bin/bash
# Round 2, run BS: encoder (BERT) flash kernels back on pointer-form tile loads -- attention tests, BERT records.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_layer.py -k "flash or attention or encoder or bert" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2bs_tests.log 2>&1 || { tail -40 gpurun_out/r2bs_tests.log; exit 1; }
tail -1 gpurun_out/r2bs_tests.log
timeout -k 10 240 python scripts/bench_bert.py --seq 512 --batch 16 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2bs_bert_seq512_b16.json || exit 1
cut -c1-140 gpurun_out/r2bs_bert_seq512_b16.json
timeout -k 10 240 python scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2bs_bert_seq128_b64.json || exit 1
cut -c1-140 gpurun_out/r2bs_bert_seq128_b64.json
