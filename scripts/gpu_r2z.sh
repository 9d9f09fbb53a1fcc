#!/bin/bash
# Round 2, run Z: flash kernels after the compile-time layout switch -- tests, attention timing,
# kernel profile of the causal flash at the 20B shape, BERT and the headline bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_sparse_flash.py tests/test_transformer_layer.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r2z_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2z_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python scripts/bench_attn.py --D 96 --flash-only > gpurun_out/r2z_attn.jsonl 2>&1 || { tail -5 gpurun_out/r2z_attn.jsonl; exit 1; }
cat gpurun_out/r2z_attn.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2z -o attn -- python $GRAFT_REPO_ROOT/scripts/bench_attn.py --D 96 --flash-only > /dev/null 2>&1 && echo profiled
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2z_bert_s128.json && cut -c1-140 gpurun_out/r2z_bert_s128.json
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2z_bench.json 2> gpurun_out/r2z_bench.log || { tail -20 gpurun_out/r2z_bench.log; exit 1; }
tail -c 700 gpurun_out/r2z_bench.json | head -c 250
exit $rc
