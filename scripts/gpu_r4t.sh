#!/bin/bash
# In-extension (torch's hipBLASLt) sweep at the BERT-Large (8192 tokens), GPT-NeoX 1.3B (32768 tokens) and
# GPT-NeoX-20B N>=2 (16384 tokens) shapes.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
layer() { echo "$4:$1:$2:$3 dgrad:$1:$2:$3 wgrad:$1:$2:$3 wgradT:$1:$2:$3"; }
PB=""
for nk in "3072 1024" "1024 1024" "4096 1024" "1024 4096"; do set -- $nk; PB="$PB $(layer 8192 $1 $2 fwdb)"; done
P13=""
for nk in "6144 2048" "2048 2048" "8192 2048" "2048 8192"; do set -- $nk; P13="$P13 $(layer 32768 $1 $2 fwdb)"; done
P16=""
for nk in "18432 6144" "6144 6144" "24576 6144" "6144 24576"; do set -- $nk; P16="$P16 $(layer 16384 $1 $2 fwdb)"; done
rm -f gpurun_out/r4t_sweep_*.jsonl
timeout -k 10 400 python -u scripts/lt_sweep.py gpurun_out/r4t_sweep_bert.jsonl $PB > gpurun_out/r4t_bert.log 2>&1 || { tail -20 gpurun_out/r4t_bert.log; exit 1; }
grep "TF/s" gpurun_out/r4t_bert.log
timeout -k 10 500 python -u scripts/lt_sweep.py gpurun_out/r4t_sweep_13b.jsonl $P13 > gpurun_out/r4t_13b.log 2>&1 || { tail -20 gpurun_out/r4t_13b.log; exit 1; }
grep "TF/s" gpurun_out/r4t_13b.log
timeout -k 10 500 python -u scripts/lt_sweep.py gpurun_out/r4t_sweep_20b16k.jsonl $P16 > gpurun_out/r4t_20b16k.log 2>&1 || { tail -20 gpurun_out/r4t_20b16k.log; exit 1; }
grep "TF/s" gpurun_out/r4t_20b16k.log
echo done
