#!/bin/bash
# Full GPU suite on the round-4 tree, smoke(), rotary bench at both NeoX shapes, the N=1 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4f_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4f_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { tail -30 gpurun_out/r4f_smoke.log; exit 1; }
tail -1 gpurun_out/r4f_smoke.log
timeout -k 10 200 python scripts/bench_rotary.py --shape 4,2048,64,96,24 > gpurun_out/r4f_rotary.jsonl 2> gpurun_out/r4f_rotary.log || { tail -20 gpurun_out/r4f_rotary.log; exit 1; }
timeout -k 10 200 python scripts/bench_rotary.py --shape 16,2048,16,128,32 >> gpurun_out/r4f_rotary.jsonl 2>> gpurun_out/r4f_rotary.log || { tail -20 gpurun_out/r4f_rotary.log; exit 1; }
cat gpurun_out/r4f_rotary.jsonl
timeout -k 10 300 python bench.py --model gpt-neox-1.3b --zero 2 --steps 20 --warmup 5 > gpurun_out/r4f_13b.json 2> gpurun_out/r4f_13b.log || { tail -30 gpurun_out/r4f_13b.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4f_13b.json
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.log || { tail -30 gpurun_out/r4f_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4f_bench.json
echo done
