#!/bin/bash
# HIP-graph capture of the BERT encoder (device RNG dropout): graph tests, BERT A/B graphs on/off (same box,
# 40 timed steps), then the whole GPU suite, smoke and the 20B N=1 bench on this tree.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_hip_graphs_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "graph or rng or dropout or encoder or transformer" > gpurun_out/r3t_graph_tests.log 2>&1 || { tail -40 gpurun_out/r3t_graph_tests.log; exit 1; }
tail -1 gpurun_out/r3t_graph_tests.log
B="python scripts/bench_bert.py --steps 40 --warmup 10"
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  for hg in on off on; do
    timeout -k 10 240 $B --seq $seq --batch $bs --hip-graphs $hg > gpurun_out/r3t_${seq}_g$hg.json 2> gpurun_out/r3t_${seq}_g$hg.log || { tail -30 gpurun_out/r3t_${seq}_g$hg.log; exit 1; }
    echo "bert $seq graphs=$hg $(grep -o '"value": [0-9.]*' gpurun_out/r3t_${seq}_g$hg.json)"
  done
done
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3t_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3t_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3t_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3t_smoke.log 2>&1 || { tail -30 gpurun_out/r3t_smoke.log; exit 1; }
tail -1 gpurun_out/r3t_smoke.log
timeout -k 10 420 python bench.py > gpurun_out/r3t_bench.json 2> gpurun_out/r3t_bench.log || { tail -30 gpurun_out/r3t_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3t_bench.json
