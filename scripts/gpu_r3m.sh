#!/bin/bash
# 20B: where the per-micro-batch bf16 fills come from (torch profiler with python stacks, 8 layers),
# then the full N=1 bench with the overlapped Adam on all CUs vs a CU-masked side stream (same box).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
DSA_PROFILE_STACK=1 timeout -k 10 300 python bench.py --layers 8 --steps 2 --warmup 2 --profile-steps 1 > gpurun_out/r3m_l8.json 2> gpurun_out/r3m_l8.log || { tail -30 gpurun_out/r3m_l8.log; exit 1; }
cp gpurun_out/torch_profile.txt gpurun_out/r3m_torch_profile_l8.txt
grep -c "" gpurun_out/r3m_torch_profile_l8.txt
for c in 0 32 0 32; do
  DSA_OVERLAP_CUS=$c timeout -k 10 420 python bench.py --steps 6 --warmup 3 > gpurun_out/r3m_bench_cu$c.json 2> gpurun_out/r3m_bench_cu$c.log || { tail -30 gpurun_out/r3m_bench_cu$c.log; exit 1; }
  echo "cus=$c $(grep -o '"value": [0-9.]*' gpurun_out/r3m_bench_cu$c.json)"
done
