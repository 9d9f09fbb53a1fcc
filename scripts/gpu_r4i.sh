#!/bin/bash
# Exhaustive hipBLASLt sweep of the backward layouts at the GPT-NeoX-20B (8192 tokens) and BERT-Large shapes.
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r4i_lt_sweep.jsonl
: > $out
for shp in "8192 18432 6144" "8192 6144 6144" "8192 24576 6144" "8192 6144 24576"; do
  for lay in fwd dgrad wgrad wgradT; do
    timeout -k 10 120 ./build_tools/lt_sweep $lay $shp 4 >> $out 2>> gpurun_out/r4i_lt_sweep.err || { echo "fail $lay $shp"; tail -5 gpurun_out/r4i_lt_sweep.err; exit 1; }
    tail -1 $out | cut -c1-220
  done
done
for shp in "8192 3072 1024" "8192 1024 1024" "8192 4096 1024" "8192 1024 4096"; do
  for lay in wgrad wgradT; do
    timeout -k 10 120 ./build_tools/lt_sweep $lay $shp 4 >> $out 2>> gpurun_out/r4i_lt_sweep.err || { echo "fail $lay $shp"; exit 1; }
    tail -1 $out | cut -c1-220
  done
done
echo done
