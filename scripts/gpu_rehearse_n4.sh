#!/bin/bash
# N=4 memory-plan rehearsal on one GPU (4 gloo ranks x 1/4 HBM, 11 of 44 layers), progress per micro-batch phase.
export TMPDIR=/tmp
mkdir -p gpurun_out
DSA_MEMTRACE=1 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29704 bench.py --gpus 4 --dist-backend gloo --layers 11 --steps 1 --warmup 1 \
  > gpurun_out/reh20b_n4.json 2> gpurun_out/reh20b_n4.log || { grep -v "^\[rank[123]\]" gpurun_out/reh20b_n4.log | tail -30; exit 1; }
grep "\[bench\]" gpurun_out/reh20b_n4.log
tail -c 1500 gpurun_out/reh20b_n4.json
