#!/bin/bash
# Kernel profile of the flagship bench, then a 2-rank memory rehearsal of the N=2 plan.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
bash scripts/gpu_prof.sh && bash scripts/gpu_rehearse_nx.sh 2
