#!/bin/bash
# hipBLASLt sweep with solution names: GPT-NeoX-20B (8192 and 16384 tokens, LM head), GPT-NeoX 1.3B
# (32768 tokens), BERT-Large (8192 tokens); table built on the box; wrapper debug; 20B N=1 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
sweep() {  # tag, problems...
  tag=$1; shift
  timeout -k 10 500 ./build_tools/lt_sweep "$@" > gpurun_out/r4k_lt_sweep_$tag.jsonl 2> gpurun_out/r4k_lt_sweep_$tag.err || { echo "fail $tag"; tail -5 gpurun_out/r4k_lt_sweep_$tag.err; return 1; }
  cut -c1-150 gpurun_out/r4k_lt_sweep_$tag.jsonl
}
layer() {  # M N K bias-layout
  echo "$4:$1:$2:$3 dgrad:$1:$2:$3 wgrad:$1:$2:$3 wgradT:$1:$2:$3"
}
P8=""; P16=""
for nk in "18432 6144" "6144 6144" "24576 6144" "6144 24576"; do
  set -- $nk
  P8="$P8 $(layer 8192 $1 $2 fwdb)"; P16="$P16 $(layer 16384 $1 $2 fwdb)"
done
PH="$(layer 8192 50432 6144 fwd) $(layer 16384 50432 6144 fwd)"
P13=""
for nk in "6144 2048" "2048 2048" "8192 2048" "2048 8192"; do
  set -- $nk
  P13="$P13 $(layer 32768 $1 $2 fwdb)"
done
P13="$P13 $(layer 32768 50304 2048 fwd)"
PB=""
for nk in "3072 1024" "1024 1024" "4096 1024" "1024 4096"; do
  set -- $nk
  PB="$PB fwdb:8192:$1:$2 dgrad:8192:$1:$2 wgrad:8192:$1:$2"
done
sweep neox20b_m8192 $P8 && sweep neox20b_head $PH && sweep neox20b_m16384 $P16 && sweep neox13b_m32768 $P13 && sweep bert_m8192 $PB || exit 1
python scripts/make_lt_table.py gpurun_out/r4k_lt_sweep_*.jsonl && cp deeperspeed_amd/ops/lt_table.json gpurun_out/lt_table.json || exit 1
DSA_LT=1 DSA_LT_DEBUG=1 timeout -k 10 300 python scripts/lt_debug.py > gpurun_out/r4k_debug.log 2>&1 || { tail -20 gpurun_out/r4k_debug.log; exit 1; }
grep "registered names\|finalist" gpurun_out/r4k_debug.log | cut -c1-160
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4k_bench_$tag.json 2> gpurun_out/r4k_bench_$tag.log || { tail -30 gpurun_out/r4k_bench_$tag.log; return 1; }
  python - gpurun_out/r4k_bench_$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = r["config"]
print(sys.argv[2], r["value"], r["ms_per_step"], "attn", c["stashed_attention_layers"], "mlp", c["stashed_mlp_layers"],
      "peak", c["peak_hbm_gib"], "lt", c.get("lt_gemm"))
PY
  grep "warmup 2" gpurun_out/r4k_bench_$tag.log
}
run lt DSA_LT=1 && run nolt DSA_LT=0
echo done
