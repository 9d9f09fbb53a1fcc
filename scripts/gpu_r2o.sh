#!/bin/bash
# Round 2, run O: headline bench with the stash safety check; N=2 / N=4 memory rehearsals of the
# sharded bench path (gloo ranks sharing the card, 1/N of HBM and 44/N layers each).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2o_bench.json 2> gpurun_out/r2o_bench.log || { tail -30 gpurun_out/r2o_bench.log; exit 1; }
grep "\[bench\]" gpurun_out/r2o_bench.log; tail -c 300 gpurun_out/r2o_bench.json
for n in 2 4; do
  layers=$((44 / n))
  DSA_MEMTRACE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --dist-backend gloo --layers $layers --steps 1 --warmup 1 \
    > gpurun_out/r2o_reh_n$n.json 2> gpurun_out/r2o_reh_n$n.log || { grep -v "mem after" gpurun_out/r2o_reh_n$n.log | tail -30; exit 1; }
  grep "\[bench\]" gpurun_out/r2o_reh_n$n.log | grep -v "mem after" | head -20
  cat gpurun_out/r2o_reh_n$n.json
done
