#!/bin/bash
# End-of-round validation of the final round-4 tree: full GPU test suite, smoke(), the default bench
# (driver contract), BERT-Large seq 128 / 512, GPT-NeoX 1.3B ZeRO-2, and a timed kernel profile of the
# default 20B N=1 step.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { tail -60 gpurun_out/final_gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.log || { tail -30 gpurun_out/final_bench.log; exit 1; }
cut -c1-300 gpurun_out/final_bench.json
timeout -k 10 300 python scripts/bench_bert.py --seq 128 --batch 64 --steps 40 --warmup 10 > gpurun_out/final_bert128.json 2> gpurun_out/final_bert128.log || { tail -20 gpurun_out/final_bert128.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/final_bert128.json
timeout -k 10 300 python scripts/bench_bert.py --seq 512 --batch 16 --steps 40 --warmup 10 > gpurun_out/final_bert512.json 2> gpurun_out/final_bert512.log || { tail -20 gpurun_out/final_bert512.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/final_bert512.json
timeout -k 10 400 python bench.py --model gpt-neox-1.3b --zero 2 --steps 20 --warmup 5 > gpurun_out/final_13b.json 2> gpurun_out/final_13b.log || { tail -20 gpurun_out/final_13b.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/final_13b.json
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/final_prof -o k --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/final_prof.json 2> $R/gpurun_out/final_prof.log || { echo "rocprof failed"; tail -20 $R/gpurun_out/final_prof.log; exit 1; }
cd $R
grep -o '"value": [0-9.]*' gpurun_out/final_prof.json
echo done
