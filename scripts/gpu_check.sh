#!/bin/bash
# GPU validation: runs steps in order, stops at the first crash/timeout (never retries).
# usage: scripts/gpu_check.sh "<name> <timeout_s> <cmd...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%% *}; rest=${spec#* }; tmo=${rest%% *}; cmd=${rest#* }
  echo "=== $name (timeout ${tmo}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc elapsed=$(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 4 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;  # ok / test failures: continue with the next step
    *) echo "stopping after rc=$rc"; exit $rc ;;
  esac
done
