#!/bin/bash
# Round 2, run BR: final-tree kernel profile of the 20B step + BERT-Large records.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 240 python scripts/bench_bert.py --seq 128 --batch 64 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2br_bert_seq128_b64.json || exit 1
cut -c1-160 gpurun_out/r2br_bert_seq128_b64.json
timeout -k 10 240 python scripts/bench_bert.py --seq 512 --batch 16 --steps 20 --warmup 5 2>/dev/null | grep '^{"metric' > gpurun_out/r2br_bert_seq512_b16.json || exit 1
cut -c1-160 gpurun_out/r2br_bert_seq512_b16.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2br -o neox -- python $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r2br_prof.json 2> $R/gpurun_out/r2br_prof.log || { tail -20 $R/gpurun_out/r2br_prof.log; exit 1; }
echo profiled
