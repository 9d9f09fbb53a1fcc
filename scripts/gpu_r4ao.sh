#!/bin/bash
# r4ao: BERT-Large weight-gradient formulation A/B on one box: split-K (default) vs ONE unsplit GEMM
# (DSA_WGRAD_SPLIT=1) vs the measured TN solutions (DSA_LT_WGRAD=1)
set -o pipefail
mkdir -p gpurun_out/r4ao
cd /root/repo
run() {  # name seq batch env...
  local name=$1 seq=$2 b=$3; shift 3
  env "$@" timeout -k 10 300 python -u scripts/bench_bert.py --seq $seq --batch $b --steps 40 --warmup 10 > gpurun_out/r4ao/$name.json 2> gpurun_out/r4ao/$name.err || exit 1
  grep -o '"value": [0-9.]*' gpurun_out/r4ao/$name.json
}
run s128_split4 128 64 DSA_NOP=1
run s128_unsplit 128 64 DSA_WGRAD_SPLIT=1
run s128_ltwgrad 128 64 DSA_LT_WGRAD=1
run s128_split4_b 128 64 DSA_NOP=1
run s512_split4 512 16 DSA_NOP=1
run s512_unsplit 512 16 DSA_WGRAD_SPLIT=1
