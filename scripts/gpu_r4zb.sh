#!/bin/bash
# GRBM_GUI_ACTIVE (kernel busy cycles) of the D = 128 flash kernels, to compare with r4z (pad 8).
export TMPDIR=/tmp
mkdir -p gpurun_out/r4zb_pmc
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES -d $R/gpurun_out/r4zb_pmc/d128 -o run --output-format csv -- python $R/scripts/bench_attn.py --D 128 96 --iters 3 --flash-only > $R/gpurun_out/r4zb_pmc/d128.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/r4zb_pmc/d128.log; exit 1; }
echo done
