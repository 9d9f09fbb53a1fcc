#!/bin/bash
# Overlapped optimizer step on/off at 20B N=1 with host moments (LM head + last layer), one box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/r4ab_$tag.json 2> gpurun_out/r4ab_$tag.log || { tail -30 gpurun_out/r4ab_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4ab_$tag.json) $(grep 'warmup 2' gpurun_out/r4ab_$tag.log | grep -o 'fwd=.*step=[0-9.]*s')"
}
run ov1 DSA_OVERLAP_STEP=1 && run ov0 DSA_OVERLAP_STEP=0 && run ov1b DSA_OVERLAP_STEP=1 && run ov0b DSA_OVERLAP_STEP=0 || exit 1
echo done
