#!/bin/bash
# Round 2, run AD: permlane32_swap row reductions in the flash forward kernels -- tests + timing.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_sparse_flash.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r2ad_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2ad_tests.log
[ $rc -le 1 ] || exit $rc
for i in 1 2 3; do timeout -k 10 200 python scripts/bench_attn.py --D 96 64 --flash-only 2>/dev/null | grep '^{' ; done
timeout -k 10 240 python scripts/bench_bert.py --seq 512 --batch 16 --steps 10 --warmup 3 2>/dev/null | grep '^{"metric' | cut -c1-140
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2ad_bench.json 2> gpurun_out/r2ad_bench.log || { tail -20 gpurun_out/r2ad_bench.log; exit 1; }
wc -l gpurun_out/r2ad_bench.json; cut -c1-200 gpurun_out/r2ad_bench.json
exit $rc
