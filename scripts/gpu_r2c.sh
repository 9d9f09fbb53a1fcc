#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 60 python scripts/diag_rccl_stash.py > gpurun_out/stash_default.log 2>&1 && cat gpurun_out/stash_default.log | grep -v Warn
TORCH_NCCL_AVOID_RECORD_STREAMS=0 MASTER_PORT=29624 timeout -k 10 60 python scripts/diag_rccl_stash.py 2>&1 | grep -v Warn
TORCH_NCCL_AVOID_RECORD_STREAMS=1 MASTER_PORT=29625 timeout -k 10 60 python scripts/diag_rccl_stash.py 2>&1 | grep -v Warn
timeout -k 10 240 python scripts/diag_zero3_mem.py --layers 6 --force-sharded > gpurun_out/diag_sharded.log 2>&1; r=$?; grep -v "config.py\|INFO" gpurun_out/diag_sharded.log | grep "GiB"; exit $r
