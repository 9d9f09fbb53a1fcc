#!/bin/bash
# Host-moments Adam on the step stream after the HBM groups + narrow D2H kernel: exactness, copy probe,
# 20B N=1 A/B against the first version, and a timed trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_host_moments_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -1 gpurun_out/r4s_tests.log
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4s_bench_$tag.json 2> gpurun_out/r4s_bench_$tag.log || { tail -30 gpurun_out/r4s_bench_$tag.log; return 1; }
  python - gpurun_out/r4s_bench_$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = r["config"]
print(sys.argv[2], r["value"], r["ms_per_step"], "attn", c["stashed_attention_layers"], "mlp", c["stashed_mlp_layers"],
      "peak", c["peak_hbm_gib"])
PY
}
run ded16 && run shared_blit DSA_DEDICATED_STREAMS=0 DSA_HOST_D2H_WGS=0 && run ded_blit DSA_HOST_D2H_WGS=0 && run ded16_side DSA_HOST_STEP_MODE=side && run ded16b || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r4s_prof -o k --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/r4s_prof.json 2> $R/gpurun_out/r4s_prof.log || { echo "rocprof failed"; tail -20 $R/gpurun_out/r4s_prof.log; exit 1; }
cd $R
grep -o '"value": [0-9.]*' gpurun_out/r4s_prof.json
echo done
