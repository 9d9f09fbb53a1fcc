#!/bin/bash
# Two-stream dgrad / wgrad for small linears (BERT-Large A/B), gathered-sparse contiguous fast path,
# NeoX 1.3B (16x1) timed kernel profile.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_par_wgrad_gpu.py tests/test_sparse_flash.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1 || { tail -40 gpurun_out/r4e_tests.log; exit 1; }
tail -1 gpurun_out/r4e_tests.log
B="python scripts/bench_bert.py --steps 40 --warmup 10"
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  for pw in 0 1 0 1; do
    DSA_PAR_WGRAD=$pw timeout -k 10 200 $B --seq $seq --batch $bs > gpurun_out/r4e_${seq}_pw$pw.json 2> gpurun_out/r4e_${seq}_pw$pw.log || { tail -30 gpurun_out/r4e_${seq}_pw$pw.log; exit 1; }
    echo "bert $seq par_wgrad=$pw $(grep -o '"value": [0-9.]*' gpurun_out/r4e_${seq}_pw$pw.json)"
  done
done
timeout -k 10 200 python scripts/bench_sparse_attn.py --mode bigbird --block 64 > gpurun_out/r4e_bigbird64.jsonl 2> gpurun_out/r4e_sparse.log || { tail -20 gpurun_out/r4e_sparse.log; exit 1; }
cat gpurun_out/r4e_bigbird64.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4e_13b -o k --output-format csv -- python3 $R/bench.py --model gpt-neox-1.3b --zero 2 --steps 5 --warmup 3 > $R/gpurun_out/r4e_13b_prof.json 2> $R/gpurun_out/r4e_13b_prof.log || { echo "1.3b rocprof failed"; tail -20 $R/gpurun_out/r4e_13b_prof.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r4e_13b_prof.json
echo done
