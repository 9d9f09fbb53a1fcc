#!/bin/bash
# PMC counters of the flash-attention kernels (20B shape, D=96), one rocprofv3 pass per counter group.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $R/gpurun_out/pmc/list.txt && printf "%s " "$c"; done; }
P1=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS)
P2=$(have SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE)
P3=$(have SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_COUNT)
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  [ -z "$P" ] && continue
  echo "pass $i: $P"
  timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python $R/scripts/bench_attn.py --D 96 --iters 3 --flash-only > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
done
ls -R $R/gpurun_out/pmc | head -30
