#!/bin/bash
# Selective recompute stash for block-sparse attention: exactness, then 20B BigBird seq 8192 (stash on / off).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_neox_stash_gpu.py tests/test_sparse_flash.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4ad_tests.log 2>&1 || { tail -40 gpurun_out/r4ad_tests.log; exit 1; }
tail -1 gpurun_out/r4ad_tests.log
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 600 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --steps 6 --warmup 3 > gpurun_out/r4ad_$tag.json 2> gpurun_out/r4ad_$tag.log || { tail -30 gpurun_out/r4ad_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"stashed_attention_layers": [0-9]*\|"stashed_mlp_layers": [0-9]*\|"peak_hbm_gib": [0-9.]*' gpurun_out/r4ad_$tag.json | tr '\n' ' ')"
}
run stash && run nostash DSA_STASH=0 || exit 1
echo done
