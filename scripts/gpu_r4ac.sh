#!/bin/bash
# Host-moments D2H: blit kernel (256 workgroups) vs narrow copy kernel, pooled queues, 20B N=1.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/r4ac_$tag.json 2> gpurun_out/r4ac_$tag.log || { tail -30 gpurun_out/r4ac_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4ac_$tag.json) $(grep 'warmup 2' gpurun_out/r4ac_$tag.log | grep -o 'fwd=.*step=[0-9.]*s')"
}
run blit DSA_HOST_D2H_WGS=0 && run n16 DSA_HOST_D2H_WGS=16 && run blitb DSA_HOST_D2H_WGS=0 && run n16b DSA_HOST_D2H_WGS=16 && run n32 DSA_HOST_D2H_WGS=32 || exit 1
echo done
