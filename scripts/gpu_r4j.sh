#!/bin/bash
# Measured hipBLASLt solutions (ops/lt_tune.py): numerics, then the 20B N=1 bench A/B on one box,
# together with the host-moments / MLP-stash variants.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_lt_tune_gpu.py tests/test_host_moments_gpu.py tests/test_neox_stash_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1 || { tail -40 gpurun_out/r4j_tests.log; exit 1; }
tail -1 gpurun_out/r4j_tests.log
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4j_bench_$tag.json 2> gpurun_out/r4j_bench_$tag.log || { tail -30 gpurun_out/r4j_bench_$tag.log; return 1; }
  python - gpurun_out/r4j_bench_$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = r["config"]
print(sys.argv[2], r["value"], r["ms_per_step"], "attn", c["stashed_attention_layers"], "mlp", c["stashed_mlp_layers"],
      "peak", c["peak_hbm_gib"], "hm", c["host_moments_params"], "lt", c.get("lt_gemm"))
PY
}
run lt_hm_mlp DSA_LT=1 && run nolt_hm_mlp DSA_LT=0 && run lt_base DSA_LT=1 DSA_MLP_STASH=0 DSA_BENCH_HOST_MOMENTS=0 && run nolt_base DSA_LT=0 DSA_MLP_STASH=0 DSA_BENCH_HOST_MOMENTS=0
echo done
