#!/bin/bash
# Offloaded optimizer steps with copy streams on dedicated hardware queues (default) vs pooled queues.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_host_moments_gpu.py tests/test_engine_gpu.py -x -q -m gpu -k "offload or moments" --timeout 200 --timeout-method thread > gpurun_out/r4ag_tests.log 2>&1 || { tail -40 gpurun_out/r4ag_tests.log; exit 1; }
tail -1 gpurun_out/r4ag_tests.log
run() {  # tag, args..., then env via E
  tag=$1; shift
  env $E timeout -k 10 900 python bench.py "$@" > gpurun_out/r4ag_$tag.json 2> gpurun_out/r4ag_$tag.log || { tail -30 gpurun_out/r4ag_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4ag_$tag.json) $(grep 'warmup 1 ' gpurun_out/r4ag_$tag.log | grep -o 'step=[0-9.]*s')"
}
E="" run 30b_ded --hidden 7168 --layers 48 --offload moments --steps 3 --warmup 2 || exit 1
E="DSA_OFFLOAD_DEDICATED_STREAMS=0" run 30b_pool --hidden 7168 --layers 48 --offload moments --steps 3 --warmup 2 || exit 1
E="" run 67b_ded --model gpt3-6.7b --offload all --ckpt on --steps 4 --warmup 2 || exit 1
E="DSA_OFFLOAD_DEDICATED_STREAMS=0" run 67b_pool --model gpt3-6.7b --offload all --ckpt on --steps 4 --warmup 2 || exit 1
echo done
