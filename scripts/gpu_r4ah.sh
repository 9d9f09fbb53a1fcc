#!/bin/bash
# states="moments" offload: 3 vs 6 device staging slots (30.3B, dedicated copy queues).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {
  tag=$1; shift
  env $E timeout -k 10 900 python bench.py --hidden 7168 --layers 48 --offload moments --steps 3 --warmup 2 > gpurun_out/r4ah_$tag.json 2> gpurun_out/r4ah_$tag.log || { tail -30 gpurun_out/r4ah_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4ah_$tag.json) $(grep 'warmup 1 ' gpurun_out/r4ah_$tag.log | grep -o 'step=[0-9.]*s')"
}
E="DSA_OFFLOAD_NBUF=6" run nbuf6 && E="DSA_OFFLOAD_NBUF=3" run nbuf3 || exit 1
echo done
