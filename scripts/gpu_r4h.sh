#!/bin/bash
# Host-moments parameter groups: exactness tests, then the 20B N=1 bench A/B on one box
# (LM head + last 2 layers' Adam moments in pinned host memory vs all in HBM).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_host_moments_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1 || { tail -40 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
for hm in auto 0; do
  timeout -k 10 420 python bench.py --steps 6 --warmup 3 --host-moments-layers $hm > gpurun_out/r4h_bench_hm$hm.json 2> gpurun_out/r4h_bench_hm$hm.log || { tail -30 gpurun_out/r4h_bench_hm$hm.log; exit 1; }
  echo "host_moments=$hm $(grep -o '"value": [0-9.]*' gpurun_out/r4h_bench_hm$hm.json) $(grep -o '"stashed_attention_layers": [0-9]*' gpurun_out/r4h_bench_hm$hm.json) $(grep -o '"peak_hbm_gib": [0-9.]*' gpurun_out/r4h_bench_hm$hm.json)"
done
echo done
