#!/bin/bash
# BASELINE rows 9 / 13: 13B model on one GPU with ZeRO-Offload (optimizer states on the CPU), ZeRO-3 vs ZeRO-2.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {
  tag=$1; shift
  timeout -k 10 900 python bench.py "$@" > gpurun_out/r4ak_$tag.json 2> gpurun_out/r4ak_$tag.log || { tail -30 gpurun_out/r4ak_$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"model_tflops_per_gpu": [0-9.]*\|"params_per_gpu": [0-9.]*\|"peak_hbm_gib": [0-9.]*' gpurun_out/r4ak_$tag.json | tr '\n' ' ')"
}
run z3_13b --hidden 5120 --layers 40 --offload all --ckpt on --steps 3 --warmup 2 || exit 1
run z2_13b --hidden 5120 --layers 40 --offload all --ckpt on --zero 2 --steps 3 --warmup 2 || exit 1
echo done
