#!/bin/bash
# Round 2, run BK: selective-recompute stash margin A/B on one box (3 GiB default vs 2 GiB), alternating.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for rep in 1 2; do
  for m in 2 3; do
    DSA_STASH_MARGIN_GIB=$m timeout -k 10 400 python bench.py > gpurun_out/r2bk_m$m.$rep.json 2> gpurun_out/r2bk_m$m.$rep.log || { tail -20 gpurun_out/r2bk_m$m.$rep.log; exit 1; }
    echo "margin=$m rep=$rep $(cut -c60-125 gpurun_out/r2bk_m$m.$rep.json) $(grep -o 'selective recompute: [0-9]*/44' gpurun_out/r2bk_m$m.$rep.log) $(grep -o 'stash safety.*' gpurun_out/r2bk_m$m.$rep.log | head -1)"
  done
done
