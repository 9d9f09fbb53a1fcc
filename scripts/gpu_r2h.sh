#!/bin/bash
# Round 2, run H: BASELINE config 5 on one MI355X -- GPT-NeoX-20B, seq 8192, block-sparse (BigBird,
# fused LUT kernel) vs dense flash at the same shape; then the ZeRO-Infinity NVMe path with
# block-sparse attention on a 5.5B NeoX-style model (fp32 master + moments on the box's disk:
# 66 GB; the full 20B would need 246 GB of NVMe and the box has 79 GB).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 500 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --block 64 --steps 2 --warmup 2 \
  > gpurun_out/r2h_20b_bigbird_s8k.json 2> gpurun_out/r2h_20b_bigbird_s8k.log || { grep -v config.py gpurun_out/r2h_20b_bigbird_s8k.log | tail -20; exit 1; }
grep "\[bench\]" gpurun_out/r2h_20b_bigbird_s8k.log; tail -c 500 gpurun_out/r2h_20b_bigbird_s8k.json
timeout -k 10 500 python bench.py --seq 8192 --micro-batch 1 --grad-accum 4 --steps 2 --warmup 2 \
  > gpurun_out/r2h_20b_dense_s8k.json 2> gpurun_out/r2h_20b_dense_s8k.log || { grep -v config.py gpurun_out/r2h_20b_dense_s8k.log | tail -20; exit 1; }
grep "\[bench\]" gpurun_out/r2h_20b_dense_s8k.log; tail -c 500 gpurun_out/r2h_20b_dense_s8k.json
df -h /tmp
timeout -k 10 600 python bench.py --hidden 4096 --layers 24 --seq 8192 --micro-batch 1 --grad-accum 4 --sparse bigbird --block 64 \
  --offload nvme --nvme-path /tmp/dsa_nvme --steps 1 --warmup 1 \
  > gpurun_out/r2h_5b_nvme_bigbird_s8k.json 2> gpurun_out/r2h_5b_nvme_bigbird_s8k.log || { grep -v config.py gpurun_out/r2h_5b_nvme_bigbird_s8k.log | tail -20; exit 1; }
grep "\[bench\]" gpurun_out/r2h_5b_nvme_bigbird_s8k.log; tail -c 700 gpurun_out/r2h_5b_nvme_bigbird_s8k.json
