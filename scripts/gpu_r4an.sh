#!/bin/bash
# r4an: the driver's N>1 launch path (torch.distributed.run, one process per rank) on the final
# round-4 tree, rehearsed with 2 and 4 ranks sharing the one GPU (gloo collectives: RCCL refuses
# two ranks on one device), 6 of the 44 GPT-NeoX-20B layers
set -o pipefail
mkdir -p gpurun_out/r4an
cd /root/repo
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n \
    bench.py --gpus $n --steps 2 --warmup 2 --layers 6 --dist-backend gloo > gpurun_out/r4an/n$n.json 2> gpurun_out/r4an/n$n.log || { tail -30 gpurun_out/r4an/n$n.log; exit 1; }
  cut -c1-400 gpurun_out/r4an/n$n.json
done
