#!/bin/bash
# Two-vector ILP in the bias+GeLU forward / backward and 3-way add kernels: kernel tests, 20B bench and its
# timed kernel profile, BERT-Large seq 128.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gelu or add3 or layernorm or embedding" > gpurun_out/r3v_tests.log 2>&1 || { tail -40 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
timeout -k 10 420 python bench.py > gpurun_out/r3v_bench.json 2> gpurun_out/r3v_bench.log || { tail -30 gpurun_out/r3v_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3v_bench.json
timeout -k 10 200 python scripts/bench_bert.py --steps 40 --warmup 10 --seq 128 --batch 64 > gpurun_out/r3v_bert128.json 2> gpurun_out/r3v_bert128.log || { tail -30 gpurun_out/r3v_bert128.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3v_bert128.json
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3v_prof20b -o neox --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r3v_prof20b.json 2> $R/gpurun_out/r3v_prof20b.log || { echo "20b rocprof failed"; tail -20 $R/gpurun_out/r3v_prof20b.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r3v_prof20b.json
