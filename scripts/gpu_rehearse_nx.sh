#!/bin/bash
# Memory-plan rehearsal of the N-GPU 20B ZeRO-3 bench on ONE GPU: N ranks (gloo) share the card,
# each gets 1/N of HBM, and the model keeps 44/N layers, so every rank's states / activations /
# retained parameters are the same fraction of its budget as on the real N-GPU node.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for n in "$@"; do
  layers=$((44 / n))
  timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --dist-backend gloo --layers $layers --steps 1 --warmup 1 \
    > gpurun_out/reh20b_n$n.json 2> gpurun_out/reh20b_n$n.log || { tail -30 gpurun_out/reh20b_n$n.log; exit 1; }
  grep "\[bench\]" gpurun_out/reh20b_n$n.log
  cat gpurun_out/reh20b_n$n.json
done
