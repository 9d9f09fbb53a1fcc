#!/bin/bash
# Current tree: GPU suite, smoke, and timed-region kernel profiles of the 20B step and BERT-Large seq 128.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3o_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3o_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3o_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3o_smoke.log 2>&1 || { tail -30 gpurun_out/r3o_smoke.log; exit 1; }
tail -1 gpurun_out/r3o_smoke.log
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3o_prof20b -o neox --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r3o_prof20b.json 2> $R/gpurun_out/r3o_prof20b.log || { echo "20b rocprof failed"; tail -20 $R/gpurun_out/r3o_prof20b.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r3o_prof20b.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3o_profbert -o bert --output-format csv -- python3 $R/scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 > $R/gpurun_out/r3o_profbert.json 2> $R/gpurun_out/r3o_profbert.log || { echo "bert rocprof failed"; tail -20 $R/gpurun_out/r3o_profbert.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/r3o_profbert.json
cd $R && timeout -k 10 200 python scripts/bench_bert.py --seq 128 --batch 64 --steps 5 --warmup 3 --torch-profile gpurun_out/r3o_bert_torchprof.txt > gpurun_out/r3o_bert_tp.json 2> gpurun_out/r3o_bert_tp.log || { tail -20 gpurun_out/r3o_bert_tp.log; exit 1; }
echo done
