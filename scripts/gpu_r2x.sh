#!/bin/bash
# Round 2, run X: same-box A/B of the fused short-sequence flash backward (BERT seq 128).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for rep in 1 2; do
  for sh in 1 0; do
    DSA_FLASH_BWD_SHORT=$sh timeout -k 10 240 python scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2x_bert_short$sh.$rep.json || exit 1
    echo "short=$sh rep=$rep $(cut -c60-140 gpurun_out/r2x_bert_short$sh.$rep.json)"
  done
done
