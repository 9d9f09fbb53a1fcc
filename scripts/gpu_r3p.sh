#!/bin/bash
# ZeRO-Infinity record with 3 timed steps: 5.2B NeoX, optimizer states on NVMe (io_uring), BigBird seq 8192.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
df -h /tmp | tail -1
timeout -k 10 1000 python bench.py --hidden 4096 --layers 24 --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --offload nvme --steps 3 --warmup 1 > gpurun_out/r3p_5b_nvme.json 2> gpurun_out/r3p_5b_nvme.log || { tail -30 gpurun_out/r3p_5b_nvme.log; exit 1; }
cat gpurun_out/r3p_5b_nvme.json
rm -rf /tmp/dsa_nvme
