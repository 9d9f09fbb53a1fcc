#!/bin/bash
# Graphed encoder with persistent, in-place-accumulated gradients: graph tests, BERT A/B graphs on/off.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_hip_graphs_gpu.py tests/test_lamb_overlap_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3u_graph_tests.log 2>&1 || { tail -40 gpurun_out/r3u_graph_tests.log; exit 1; }
tail -1 gpurun_out/r3u_graph_tests.log
B="python scripts/bench_bert.py --steps 40 --warmup 10"
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  for hg in on off on off; do
    timeout -k 10 240 $B --seq $seq --batch $bs --hip-graphs $hg > gpurun_out/r3u_${seq}_g$hg.json 2> gpurun_out/r3u_${seq}_g$hg.log || { tail -30 gpurun_out/r3u_${seq}_g$hg.log; exit 1; }
    echo "bert $seq graphs=$hg $(grep -o '"value": [0-9.]*' gpurun_out/r3u_${seq}_g$hg.json)"
  done
done
