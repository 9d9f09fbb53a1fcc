#!/bin/bash
# A/B of flash-attention forward variants at the 20B shape + the flash numerics tests.
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python scripts/bench_attn.py --D 96 64 --flash-only --iters 30 > gpurun_out/fa_new_$i.log 2>&1 || exit 1
  DSA_FLASH_FWD_V2=1 timeout -k 10 120 python scripts/bench_attn.py --D 96 64 --flash-only --iters 30 > gpurun_out/fa_old_$i.log 2>&1 || exit 1
done
grep -h '"B"' gpurun_out/fa_new_*.log; echo old; grep -h '"B"' gpurun_out/fa_old_*.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/fa_tests.log 2>&1; tail -3 gpurun_out/fa_tests.log
