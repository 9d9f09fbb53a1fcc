#!/bin/bash
# Round 3: LDS-staged, stride-aware sparse MatMul kernels and single-evaluation sparse softmax.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "sparse or rotary" tests/test_sparse_attention.py tests/test_sparse_flash.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 || { tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -1 gpurun_out/r3g_tests.log
timeout -k 10 120 python scripts/bench_rotary.py > gpurun_out/r3g_rotary.jsonl 2> gpurun_out/r3g_rotary.err || { tail -20 gpurun_out/r3g_rotary.err; exit 1; }
cat gpurun_out/r3g_rotary.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --unfused > gpurun_out/r3g_sparse.jsonl 2> gpurun_out/r3g_sparse.err || { tail -20 gpurun_out/r3g_sparse.err; exit 1; }
cat gpurun_out/r3g_sparse.jsonl
timeout -k 10 200 python scripts/bench_sparse_attn.py --unfused --seq 4096 --heads 16 --dim 64 --batch 4 --mode fixed --block 16 > gpurun_out/r3g_sparse_bert.jsonl 2> gpurun_out/r3g_sparse_bert.err || { tail -20 gpurun_out/r3g_sparse_bert.err; exit 1; }
cat gpurun_out/r3g_sparse_bert.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3g_prof -o sp --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_sparse_attn.py --iters 5 --unfused > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/r3g_prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r3g_kernel_stats.csv; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r3g_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1),'us')"
