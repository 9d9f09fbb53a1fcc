#!/bin/bash
# (1) flash-attention PMC counters on the current kernels (D=96 20B shape, D=128 1.3B shape);
# (2) 2-rank self-spawned bench rehearsal (gloo, both ranks on this one GPU) of the N>1 path.
export TMPDIR=/tmp
mkdir -p gpurun_out/r4z_pmc
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/r4z_pmc/list.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $R/gpurun_out/r4z_pmc/list.txt && printf "%s " "$c"; done; }
P1=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS)
P2=$(have SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT)
for D in 96 128; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    [ -z "$P" ] && continue
    timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/r4z_pmc/d${D}_p$i -o run --output-format csv -- python $R/scripts/bench_attn.py --D $D --iters 3 --flash-only > $R/gpurun_out/r4z_pmc/d${D}_p$i.log 2>&1 || { echo "pmc D=$D pass $i failed"; tail -5 $R/gpurun_out/r4z_pmc/d${D}_p$i.log; exit 1; }
  done
done
echo "pmc done"
cd $R
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --layers 4 --steps 2 --warmup 2 > gpurun_out/r4z_spawn2.json 2> gpurun_out/r4z_spawn2.log || { tail -30 gpurun_out/r4z_spawn2.log; exit 1; }
cut -c1-300 gpurun_out/r4z_spawn2.json
echo done
