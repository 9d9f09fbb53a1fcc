#!/bin/bash
# Round 2, run K: full GPU suite, headline bench (bound path), forced-sharded bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2k_gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r2k_gpu_tests.log
# plain test failures (rc 1) still allow the benches; a crash, abort or time limit ends the call
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2k_bench.json 2> gpurun_out/r2k_bench.log || { tail -30 gpurun_out/r2k_bench.log; exit 1; }
grep "\[bench\]" gpurun_out/r2k_bench.log; tail -c 400 gpurun_out/r2k_bench.json
timeout -k 10 400 python bench.py --steps 4 --warmup 2 --force-sharded > gpurun_out/r2k_bench_sharded.json 2> gpurun_out/r2k_bench_sharded.log || { grep -v config.py gpurun_out/r2k_bench_sharded.log | tail -30; exit 1; }
grep "\[bench\]" gpurun_out/r2k_bench_sharded.log; tail -c 400 gpurun_out/r2k_bench_sharded.json
exit $rc
