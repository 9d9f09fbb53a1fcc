#!/bin/bash
# BERT-Large split-K weight-gradient factor with fp32 partials: DSA_WGRAD_SPLIT 4 (default) vs 2, interleaved, same box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
B="python scripts/bench_bert.py --steps 40 --warmup 10"
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  for sp in 4 2 4 2; do
    DSA_WGRAD_SPLIT=$sp timeout -k 10 200 $B --seq $seq --batch $bs > gpurun_out/r3w_${seq}_s$sp.json 2> gpurun_out/r3w_${seq}_s$sp.log || { tail -30 gpurun_out/r3w_${seq}_s$sp.log; exit 1; }
    echo "bert $seq split=$sp $(grep -o '"value": [0-9.]*' gpurun_out/r3w_${seq}_s$sp.json)"
  done
done
