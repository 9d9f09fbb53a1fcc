#!/bin/bash
# Host-moments parameter groups + MLP stash: exactness tests, then the 20B N=1 bench on one box:
# host moments + MLP stash (default), host moments without MLP stash, neither.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_host_moments_gpu.py tests/test_neox_stash_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1 || { tail -40 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
run() {  # tag, env..., args...
  tag=$1; shift
  env "$@" timeout -k 10 420 python bench.py --steps 6 --warmup 3 > gpurun_out/r4h_bench_$tag.json 2> gpurun_out/r4h_bench_$tag.log || { tail -30 gpurun_out/r4h_bench_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4h_bench_$tag.json) $(grep -o '"stashed_[a-z]*_layers": [0-9]*' gpurun_out/r4h_bench_$tag.json | tr '\n' ' ') $(grep -o '"peak_hbm_gib": [0-9.]*' gpurun_out/r4h_bench_$tag.json)"
}
run hm_mlp DSA_MLP_STASH=1 && run hm_nomlp DSA_MLP_STASH=0 && run base DSA_MLP_STASH=0 DSA_BENCH_HOST_MOMENTS=0
echo done
