#!/bin/bash
# One parameterised runner for every GPU-box job (run through gpurun; chain steps with &&).
#
#   scripts/gpu.sh tests  [TIMEOUT] [paths / pytest args]  GPU tests (default: all of tests/) -> gpurun_out/tests.log
#   scripts/gpu.sh smoke                                   __graft_entry__.smoke()
#   scripts/gpu.sh bench  TAG TIMEOUT [bench.py args...]   1-rank bench -> gpurun_out/TAG.{json,log}
#   scripts/gpu.sh torchrun TAG TIMEOUT N [bench args...]  N ranks under torch.distributed.run (N ranks
#                                                          share the box's one GPU: pass --dist-backend gloo)
#   scripts/gpu.sh py     TAG TIMEOUT script.py [args...]  any python script -> gpurun_out/TAG.{json,log}
#   scripts/gpu.sh prof   TAG TIMEOUT script.py [args...]  rocprofv3 kernel trace of a python script,
#                                                          timed-region summary -> gpurun_out/TAG_kernel_stats.md
#   scripts/gpu.sh pmc    TAG TIMEOUT "CTR CTR.." script.py [args...]   one rocprofv3 counter pass
#
# Every GPU step runs under its own `timeout -k 10`, writes its output under gpurun_out/ and
# returns non-zero on failure, so a chain of steps joined with && stops at the first one that fails.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
task=$1
shift

fail() {  # print the tail of a failed step's log and propagate its status
  local rc=$1 log=$2
  echo "[gpu.sh] $task failed rc=$rc"
  tail -40 "$log"
  exit "$rc"
}

case "$task" in
  tests)
    t=${1:-900}
    shift || true
    [ $# -eq 0 ] && set -- tests
    timeout -k 10 "$t" python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread "$@" \
      > "$O/tests.log" 2>&1 || fail $? "$O/tests.log"
    tail -3 "$O/tests.log"
    ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail $? "$O/smoke.log"
    tail -2 "$O/smoke.log"
    ;;
  bench)
    tag=$1 t=$2
    shift 2
    timeout -k 10 "$t" python -u bench.py "$@" > "$O/$tag.json" 2> "$O/$tag.log" || fail $? "$O/$tag.log"
    grep "\[bench\]" "$O/$tag.log" | tail -8 || true
    cut -c1-400 "$O/$tag.json"
    ;;
  torchrun)
    tag=$1 t=$2 n=$3
    shift 3
    timeout -k 10 "$t" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $((29600 + RANDOM % 200)) bench.py --gpus "$n" "$@" > "$O/$tag.json" 2> "$O/$tag.log" \
      || fail $? "$O/$tag.log"
    grep "\[bench\]" "$O/$tag.log" | tail -8 || true
    cut -c1-400 "$O/$tag.json"
    ;;
  py)
    tag=$1 t=$2
    shift 2
    timeout -k 10 "$t" python -u "$@" > "$O/$tag.json" 2> "$O/$tag.log" || fail $? "$O/$tag.log"
    tail -c 2000 "$O/$tag.json"
    ;;
  prof)
    tag=$1 t=$2 script=$3
    shift 3
    cd /tmp
    timeout -k 10 "$t" rocprofv3 --kernel-trace -d "$O/$tag" -o k --output-format csv -- \
      python3 "$R/$script" "$@" > "$O/$tag.json" 2> "$O/$tag.log" || fail $? "$O/$tag.log"
    cd "$R"
    python scripts/prof_summary.py --timed "$(find "$O/$tag" -name '*kernel_trace.csv' | head -1)" \
      "$tag (timed region)" "$script $*" > "$O/${tag}_kernel_stats.md" || fail $? "$O/${tag}_kernel_stats.md"
    head -45 "$O/${tag}_kernel_stats.md"
    ;;
  pmc)
    tag=$1 t=$2 ctrs=$3 script=$4
    shift 4
    cd /tmp
    timeout -s KILL "$t" rocprofv3 --pmc $ctrs --kernel-trace --stats -d "$O/$tag" -o p --output-format csv -- \
      python3 "$R/$script" "$@" > "$O/$tag.out" 2> "$O/$tag.log" || fail $? "$O/$tag.log"
    cd "$R"
    echo "[gpu.sh] counters in $O/$tag"
    ;;
  *)
    echo "usage: scripts/gpu.sh {tests|smoke|bench|torchrun|py|prof|pmc} ..." >&2
    exit 2
    ;;
esac
