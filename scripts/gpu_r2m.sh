#!/bin/bash
# Round 2, run M: autotuned hipBLASLt GEMM wrapper -- tests and transformer-shape sweep.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gemm_lt_gpu.py tests/test_transformer_layer.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2m_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r2m_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm_shapes.py --model bert-large --tokens 8192 > gpurun_out/r2m_gemm_bert.jsonl 2> gpurun_out/r2m_gemm_bert.log || { tail -20 gpurun_out/r2m_gemm_bert.log; exit 1; }
timeout -k 10 300 python scripts/bench_gemm_shapes.py --model neox20b --tokens 8192 > gpurun_out/r2m_gemm_neox.jsonl 2> gpurun_out/r2m_gemm_neox.log || { tail -20 gpurun_out/r2m_gemm_neox.log; exit 1; }
echo done
exit $rc
