#!/bin/bash
# Rehearsal of the driver's multi-GPU bench configs on ONE GPU: N ranks (gloo) share the card.
#   scripts/rehearse.sh N [TIMEOUT] [CONFIGS]   -> gpurun_out/reh_n<N>_{c3,c2,c4}.{json,log}
# c3: BASELINE config 3 (ZeRO-3, measured memory fit), reduced to hidden 2048 x 4 layers
# c2: BASELINE config 2 (GPT-NeoX 1.3B ZeRO-2), 4 layers
# c4: BASELINE config 4 (GPT-3 6.7B PipelineModule PP x DP, 1-bit Adam), 4 layers, PP = N/2; the
#     bench's own 1-bit block (freeze after 16 steps, untimed warmup runs past it), so the 4 timed
#     steps are compressed ones and the record carries their losses and the "diverged" flag
# (the full-depth 20B plan per rank: bench.py --emulate-world N, profiles/r6a_emulated_world_notes.md)
set -e
n=$1
t=${2:-400}
cfgs=${3:-"c3 c2 c4"}
for c in $cfgs; do
  case $c in
    c3) scripts/gpu.sh torchrun reh_n${n}_c3 "$t" "$n" --dist-backend gloo --hidden 2048 --layers 4 --steps 2 --warmup 2 ;;
    c2) scripts/gpu.sh torchrun reh_n${n}_c2 "$t" "$n" --dist-backend gloo --model gpt-neox-1.3b --zero 2 --layers 4 \
          --steps 2 --warmup 2 ;;
    c4) scripts/gpu.sh torchrun reh_n${n}_c4 "$t" "$n" --dist-backend gloo --model gpt3-6.7b --pipe $((n / 2)) \
          --optimizer onebitadam --layers 4 --steps 4 --warmup 3 ;;
  esac
done
