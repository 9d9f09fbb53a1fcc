#!/bin/bash
# After the dedicated offload queues: full GPU test suite, smoke, NVMe 5.2B BigBird seq 8192 record.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4ai_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4ai_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4ai_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ai_smoke.log 2>&1 || { tail -30 gpurun_out/r4ai_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 700 python bench.py --hidden 4096 --layers 24 --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --offload nvme --steps 3 --warmup 1 > gpurun_out/r4ai_5b_nvme.json 2> gpurun_out/r4ai_5b_nvme.log || { tail -30 gpurun_out/r4ai_5b_nvme.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4ai_5b_nvme.json
echo done
