#!/bin/bash
# Round 2, run E: offload GPU tests, ZeRO-Offload (states all) bench serial vs pipelined on
# GPT-3 6.7B (host 12 B/param = 80 GB pinned), aio sweep on the box's local disk, and the
# peak-params run: NeoX-style 27.9B (hidden 7168, 44 layers) with the Adam moments on the host
# (207 GiB pinned) and compact master + grads in HBM.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q -k "offload or moments" --timeout 200 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1 || { tail -30 gpurun_out/r2e_tests.log; exit 1; }
tail -1 gpurun_out/r2e_tests.log
for mode in 0 1; do
  DSA_OFFLOAD_PIPELINE=$mode timeout -k 10 400 python bench.py --model gpt3-6.7b --offload all --ckpt on --steps 2 --warmup 1 \
     > gpurun_out/r2e_off_p$mode.json 2> gpurun_out/r2e_off_p$mode.log || { tail -20 gpurun_out/r2e_off_p$mode.log; exit 1; }
  grep "\[bench\]" gpurun_out/r2e_off_p$mode.log; tail -c 300 gpurun_out/r2e_off_p$mode.json
done
timeout -k 10 300 python scripts/aio_sweep.py --path /tmp/dsa_aio_sweep --mb 2048 --blocks 256,1024,4096 --qds 1,8,32 --threads 1,4 --reps 1 --psync-baseline > gpurun_out/r2e_aio_sweep.jsonl 2> gpurun_out/r2e_aio_sweep.log || { tail -20 gpurun_out/r2e_aio_sweep.log; exit 1; }
tail -3 gpurun_out/r2e_aio_sweep.jsonl
timeout -k 10 600 python bench.py --hidden 7168 --layers 44 --offload moments --steps 2 --warmup 1 \
   > gpurun_out/r2e_peak28b.json 2> gpurun_out/r2e_peak28b.log || { grep -v "config.py" gpurun_out/r2e_peak28b.log | tail -20; exit 1; }
grep "\[bench\]" gpurun_out/r2e_peak28b.log; tail -c 900 gpurun_out/r2e_peak28b.json
