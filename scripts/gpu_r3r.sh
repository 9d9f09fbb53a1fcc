#!/bin/bash
# Sync-free step: device-sorted embedding backward + bf16 LAMB step without a host read of the norm.
# Tests, BERT-Large A/B (DSA_SYNC_FREE_STEP=0 restores the host-checked LAMB step; the embedding change has no
# switch), the 20B N=1 bench, and a timed BERT trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_lamb_overlap_gpu.py -x -q --timeout 200 --timeout-method thread -k "embedding or lamb or sync_free or layernorm or transformer" > gpurun_out/r3r_tests.log 2>&1 || { tail -40 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
B="python scripts/bench_bert.py --steps 40 --warmup 10"
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  for sf in 1 0 1; do
    DSA_SYNC_FREE_STEP=$sf timeout -k 10 200 $B --seq $seq --batch $bs > gpurun_out/r3r_${seq}_sf$sf.json 2> gpurun_out/r3r_${seq}_sf$sf.log || { tail -30 gpurun_out/r3r_${seq}_sf$sf.log; exit 1; }
    echo "bert $seq sync_free=$sf $(grep -o '"value": [0-9.]*' gpurun_out/r3r_${seq}_sf$sf.json)"
  done
done
timeout -k 10 420 python bench.py --steps 6 --warmup 3 > gpurun_out/r3r_bench.json 2> gpurun_out/r3r_bench.log || { tail -30 gpurun_out/r3r_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3r_bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3r_profbert -o bert --output-format csv -- python3 $R/scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 > $R/gpurun_out/r3r_profbert.json 2> $R/gpurun_out/r3r_profbert.log || { echo "bert rocprof failed"; tail -20 $R/gpurun_out/r3r_profbert.log; exit 1; }
echo done
