#!/bin/bash
# r4ap: timed kernel profiles of BERT-Large seq 128 b64 and seq 512 b16 on the final round-4 tree
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
for cfg in "128 64" "512 16"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4ap_bert$1 -o k --output-format csv -- python3 $R/scripts/bench_bert.py --seq $1 --batch $2 --steps 20 --warmup 10 > $R/gpurun_out/r4ap_bert$1.json 2> $R/gpurun_out/r4ap_bert$1.log || { echo "bert rocprof failed"; tail -20 $R/gpurun_out/r4ap_bert$1.log; exit 1; }
  grep -o '"value": [0-9.]*' $R/gpurun_out/r4ap_bert$1.json
done
echo done
