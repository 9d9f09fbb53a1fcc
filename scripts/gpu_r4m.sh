#!/bin/bash
# hipBLASLt sweep with torch's own hipBLASLt (in-extension), GPT-NeoX-20B N=1 shapes; table built on the
# box; wrapper debug; 20B N=1 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
layer() { echo "$4:$1:$2:$3 dgrad:$1:$2:$3 wgrad:$1:$2:$3 wgradT:$1:$2:$3"; }
P=""
for nk in "18432 6144" "6144 6144" "24576 6144" "6144 24576"; do set -- $nk; P="$P $(layer 8192 $1 $2 fwdb)"; done
P="$P $(layer 8192 50432 6144 fwd)"
rm -f gpurun_out/r4m_sweep.jsonl
timeout -k 10 600 python -u scripts/lt_sweep.py gpurun_out/r4m_sweep.jsonl $P > gpurun_out/r4m_sweep.log 2>&1 || { tail -20 gpurun_out/r4m_sweep.log; exit 1; }
grep "TF/s" gpurun_out/r4m_sweep.log
python scripts/make_lt_table.py gpurun_out/r4m_sweep.jsonl && cp deeperspeed_amd/ops/lt_table.json gpurun_out/lt_table.json || exit 1
DSA_LT=1 DSA_LT_DEBUG=1 timeout -k 10 300 python scripts/lt_debug.py > gpurun_out/r4m_debug.log 2>&1 || { tail -20 gpurun_out/r4m_debug.log; exit 1; }
grep "registered names\|finalist" gpurun_out/r4m_debug.log | cut -c1-160
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4m_bench_$tag.json 2> gpurun_out/r4m_bench_$tag.log || { tail -30 gpurun_out/r4m_bench_$tag.log; return 1; }
  python - gpurun_out/r4m_bench_$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = r["config"]
print(sys.argv[2], r["value"], r["ms_per_step"], "attn", c["stashed_attention_layers"], "mlp", c["stashed_mlp_layers"],
      "peak", c["peak_hbm_gib"], "lt", c.get("lt_gemm"))
PY
  grep "warmup 2" gpurun_out/r4m_bench_$tag.log
}
run lt DSA_LT=1 && run nolt DSA_LT=0 || exit 1
# timed kernel + memory-copy trace of the default 20B N=1 step (3 timed steps)
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r4m_prof -o k --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/r4m_prof.json 2> $R/gpurun_out/r4m_prof.log || { echo "rocprof failed"; tail -20 $R/gpurun_out/r4m_prof.log; exit 1; }
cd $R
grep -o '"value": [0-9.]*' gpurun_out/r4m_prof.json
echo done
