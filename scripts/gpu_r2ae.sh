#!/bin/bash
# Round 2, run AE: peak parameters per GPU -- NeoX-style hidden 7168, 48 layers (30.3B) with the
# Adam moments in pinned host memory (8 B/param = 226 GiB of the box's ~270 GiB per-command cap).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python bench.py --hidden 7168 --layers 48 --offload moments --steps 2 --warmup 1 \
  > gpurun_out/r2ae_peak.json 2> gpurun_out/r2ae_peak.log || { tail -20 gpurun_out/r2ae_peak.log; exit 1; }
grep "\[bench\]" gpurun_out/r2ae_peak.log | head; cut -c1-400 gpurun_out/r2ae_peak.json
