#!/bin/bash
# Host-moments layer count on the 20B N=1 step: 1 / 2 (auto) / 3, interleaved on one box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4w_bench_$tag.json 2> gpurun_out/r4w_bench_$tag.log || { tail -30 gpurun_out/r4w_bench_$tag.log; return 1; }
  python - gpurun_out/r4w_bench_$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = r["config"]
print(sys.argv[2], r["value"], r["ms_per_step"], "attn", c["stashed_attention_layers"], "mlp", c["stashed_mlp_layers"],
      "peak", c["peak_hbm_gib"], "hm", c["host_moments_params"])
PY
}
run k2 && run k1 DSA_BENCH_HOST_MOMENTS=1 && run k3 DSA_BENCH_HOST_MOMENTS=3 && run k2b && run k1b DSA_BENCH_HOST_MOMENTS=1 || exit 1
echo done
