#!/bin/bash
# GEMM efficiency at M=16384 (micro-batch 8) + list of PMC counters on gfx950.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/bench_gemm_layouts.py --tokens 16384 --backends cublaslt > gpurun_out/gemm_m16k.log 2>&1 || exit 1
tail -1 gpurun_out/gemm_m16k.log
cd /tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt 2>&1
grep -c . $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt
