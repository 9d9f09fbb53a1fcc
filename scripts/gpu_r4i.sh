#!/bin/bash
# Exhaustive hipBLASLt sweep of the forward / backward GEMM layouts at the GPT-NeoX-20B shapes (8192 tokens).
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r4i_lt_sweep.jsonl
: > $out
M=8192
set -o pipefail
# fwd (+bias), dgrad after the weight transpose (TN), dgrad NN, wgrad NT, wgrad after both transposes (TN)
for nk in "18432 6144" "6144 6144" "24576 6144" "6144 24576"; do
  set -- $nk; N=$1; K=$2
  timeout -k 10 400 ./build_tools/lt_sweep fwdb:$M:$N:$K fwd:$M:$K:$N dgrad:$M:$N:$K wgrad:$M:$N:$K wgradT:$M:$N:$K >> $out 2>> gpurun_out/r4i_lt_sweep.err || { echo "fail $nk"; tail -5 gpurun_out/r4i_lt_sweep.err; exit 1; }
  tail -5 $out | cut -c1-200
done
echo done
