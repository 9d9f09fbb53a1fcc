#!/bin/bash
# Current tree: GPU suite, smoke, 20B N=1 bench, BERT-Large seq 128 / 512 (40 timed steps).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3s_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3s_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3s_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s_smoke.log 2>&1 || { tail -30 gpurun_out/r3s_smoke.log; exit 1; }
tail -1 gpurun_out/r3s_smoke.log
timeout -k 10 420 python bench.py > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.log || { tail -30 gpurun_out/r3s_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3s_bench.json
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  timeout -k 10 200 python scripts/bench_bert.py --steps 40 --warmup 10 --seq $seq --batch $bs > gpurun_out/r3s_bert$seq.json 2> gpurun_out/r3s_bert$seq.log || { tail -30 gpurun_out/r3s_bert$seq.log; exit 1; }
  echo "bert $seq $(grep -o '"value": [0-9.]*' gpurun_out/r3s_bert$seq.json)"
done
