#!/bin/bash
# Round 2, run J: N=4 memory-plan rehearsal of the 20B bench on ONE GPU (4 gloo ranks x 1/4 HBM,
# 11 of 44 layers each): the sharded ZeRO-3 path with prefetch window, buffer pool, bounded
# in-flight reductions and the planner's retention budget.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29704 bench.py --gpus 4 --dist-backend gloo --layers 11 --steps 1 --warmup 1 \
  > gpurun_out/r2j_reh_n4.json 2> gpurun_out/r2j_reh_n4.log || { grep -v "^\[rank[123]\]" gpurun_out/r2j_reh_n4.log | grep -v config.py | tail -30; exit 1; }
grep "\[bench\]" gpurun_out/r2j_reh_n4.log
tail -c 900 gpurun_out/r2j_reh_n4.json
