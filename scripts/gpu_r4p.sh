#!/bin/bash
# HBM -> pinned-host copy paths: blit kernel or DMA engine, per hipMemcpyKind and GPU_BLIT_ENGINE_TYPE.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
for bt in none 0 1 2; do
  if [ $bt = none ]; then E=""; else E="GPU_BLIT_ENGINE_TYPE=$bt"; fi
  echo "== GPU_BLIT_ENGINE_TYPE=$bt"
  env $E timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r4p_$bt -o k --output-format csv -- python3 $R/scripts/d2h_probe.py > $R/gpurun_out/r4p_$bt.log 2>&1 || { tail -20 $R/gpurun_out/r4p_$bt.log; exit 1; }
  grep "per 64 MB" $R/gpurun_out/r4p_$bt.log
  echo "copyBuffer kernels: $(grep -c copyBuffer $R/gpurun_out/r4p_$bt/k_kernel_trace.csv || true), DMA copies: $(grep -c DEVICE_TO_HOST $R/gpurun_out/r4p_$bt/k_memory_copy_trace.csv || true)"
done
echo done
