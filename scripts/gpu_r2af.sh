#!/bin/bash
# Round 2, run AF: selective-recompute stash margin A/B on one box (4 GiB default vs 3 GiB).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for m in 3 4 3; do
  DSA_STASH_MARGIN_GIB=$m timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/r2af_m$m.json 2> gpurun_out/r2af_m$m.log || { tail -20 gpurun_out/r2af_m$m.log; exit 1; }
  echo "margin=$m $(grep -o 'selective recompute: [0-9]*/44' gpurun_out/r2af_m$m.log) $(grep -o 'stash safety.*' gpurun_out/r2af_m$m.log) $(grep -o 'warmup 1.*' gpurun_out/r2af_m$m.log | grep -o 'reserved=[0-9.]* GiB') $(cut -c1-150 gpurun_out/r2af_m$m.json | grep -o '"value": [0-9.]*')"
done
