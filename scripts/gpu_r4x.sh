#!/bin/bash
# Validation of the current tree: full GPU test suite, smoke(), default bench (driver contract), and the
# LM-head-only host-moments variant.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4x_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4x_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4x_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4x_smoke.log 2>&1 || { tail -30 gpurun_out/r4x_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/r4x_bench.json 2> gpurun_out/r4x_bench.log || { tail -30 gpurun_out/r4x_bench.log; exit 1; }
cat gpurun_out/r4x_bench.json | cut -c1-400
timeout -k 10 400 python bench.py --steps 6 --warmup 3 --host-moments-layers head > gpurun_out/r4x_head.json 2> gpurun_out/r4x_head.log || { tail -30 gpurun_out/r4x_head.log; exit 1; }
grep -o '"value": [0-9.]*\|"stashed_attention_layers": [0-9]*\|"stashed_mlp_layers": [0-9]*' gpurun_out/r4x_head.json
timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4x_auto6.json 2> gpurun_out/r4x_auto6.log || { tail -30 gpurun_out/r4x_auto6.log; exit 1; }
grep -o '"value": [0-9.]*\|"stashed_attention_layers": [0-9]*\|"stashed_mlp_layers": [0-9]*' gpurun_out/r4x_auto6.json
echo done
