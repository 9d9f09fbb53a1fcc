#!/bin/bash
# Round 2, run BC: kernel profile of the 20B step after the transposing GeLU kernels, then one
# extra step under torch.profiler grouped by input shape (where the remaining adds / fills come from).
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2bc -o neox -- python $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r2bc_bench.json 2> $R/gpurun_out/r2bc_bench.log || { tail -20 $R/gpurun_out/r2bc_bench.log; exit 1; }
echo profiled
cd $R && timeout -k 10 500 python bench.py --steps 1 --warmup 2 --profile-steps 1 > gpurun_out/r2bc_torchprof.json 2> gpurun_out/r2bc_torchprof.log || { tail -20 gpurun_out/r2bc_torchprof.log; exit 1; }
echo torchprof done
