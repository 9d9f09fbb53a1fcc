#!/bin/bash
# HIP hardware queues: with GPU_MAX_HW_QUEUES=4 the compute stream shares a hardware queue with the
# optimizer-step streams, so the next forward waited for the host-moments Adam (profiles/r4n_notes.md).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 6 --warmup 3 > gpurun_out/r4o_bench_$tag.json 2> gpurun_out/r4o_bench_$tag.log || { tail -30 gpurun_out/r4o_bench_$tag.log; return 1; }
  python - gpurun_out/r4o_bench_$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = r["config"]
print(sys.argv[2], r["value"], r["ms_per_step"], "attn", c["stashed_attention_layers"], "mlp", c["stashed_mlp_layers"],
      "peak", c["peak_hbm_gib"])
PY
}
run q8 GPU_MAX_HW_QUEUES=8 && run q4 GPU_MAX_HW_QUEUES=4 && run q8b GPU_MAX_HW_QUEUES=8 && run q8_nohm GPU_MAX_HW_QUEUES=8 DSA_BENCH_HOST_MOMENTS=0 DSA_MLP_STASH=0 && run q4_nohm GPU_MAX_HW_QUEUES=4 DSA_BENCH_HOST_MOMENTS=0 DSA_MLP_STASH=0 || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r4o_prof -o k --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/r4o_prof.json 2> $R/gpurun_out/r4o_prof.log || { echo "rocprof failed"; tail -20 $R/gpurun_out/r4o_prof.log; exit 1; }
cd $R
grep -o '"value": [0-9.]*' gpurun_out/r4o_prof.json
echo done
