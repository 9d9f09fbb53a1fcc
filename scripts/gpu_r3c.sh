#!/bin/bash
# Round 3: flash backward dK/dV v3 (initial-accumulator row constants, halves-staged tiles)
# correctness + A/B against the v2 body and the one-wave-per-SIMD variant.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash" --timeout 120 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || { tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -1 gpurun_out/r3c_tests.log
for v in 2 3 31 2 3; do
  DSA_FA_DKDV=$v timeout -k 10 120 python scripts/bench_attn.py --D 96 --flash-only --iters 30 > gpurun_out/r3c_attn_$v.json 2>gpurun_out/r3c_attn_$v.err || { tail -20 gpurun_out/r3c_attn_$v.err; exit 1; }
  echo "dkdv=$v $(cat gpurun_out/r3c_attn_$v.json)"
done
