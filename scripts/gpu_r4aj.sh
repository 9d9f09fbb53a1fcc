#!/bin/bash
# BERT-Large overlapped LAMB step with the side stream on a dedicated hardware queue.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
bert() {  # tag seq batch args...
  tag=$1; seq=$2; b=$3; shift 3
  env $E timeout -k 10 300 python scripts/bench_bert.py --seq $seq --batch $b --steps 40 --warmup 10 "$@" > gpurun_out/r4aj_$tag.json 2> gpurun_out/r4aj_$tag.log || { tail -20 gpurun_out/r4aj_$tag.log; return 1; }
  echo "bert $tag $(grep -o '"value": [0-9.]*' gpurun_out/r4aj_$tag.json)"
}
E="" bert serial 128 64 && E="" bert ov_pool 128 64 --overlap-step on && E="DSA_DEDICATED_STREAMS=1" bert ov_ded 128 64 --overlap-step on || exit 1
E="" bert serial512 512 16 && E="DSA_DEDICATED_STREAMS=1" bert ov_ded512 512 16 --overlap-step on || exit 1
echo done
