#!/bin/bash
# torch.profiler op table of one 20B step (after the timed steps) + GPT-NeoX 1.3B ZeRO-2 bench (BASELINE config 2).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 500 python bench.py --steps 2 --warmup 2 --profile-steps 1 > gpurun_out/tp_bench.json 2> gpurun_out/tp_bench.log || { tail -30 gpurun_out/tp_bench.log; exit 1; }
grep metric gpurun_out/tp_bench.json | cut -c1-200
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 --steps 5 --warmup 2 > gpurun_out/b13.json 2> gpurun_out/b13.log || { tail -30 gpurun_out/b13.log; exit 1; }
grep metric gpurun_out/b13.json | cut -c1-400
