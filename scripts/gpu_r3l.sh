#!/bin/bash
# Kernel numerics after the LN-backward pipelining and the hoisted encoder key-bias loads; encoder attention
# variants at the BERT-Large shapes; BERT-Large with the overlapped LAMB step on all CUs, on a CU-masked side
# stream (32 / 64 CUs) and serial -- 40 timed steps, same box.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
# (passed in the previous call) timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "layernorm or encoder or qkv or flash or transformer" > gpurun_out/r3l_kernel_tests.log 2>&1 || { tail -40 gpurun_out/r3l_kernel_tests.log; exit 1; }
# tail -2 gpurun_out/r3l_kernel_tests.log
timeout -k 10 200 python scripts/bench_encoder_attn.py > gpurun_out/r3l_encoder_attn.jsonl 2> gpurun_out/r3l_encoder_attn.log || { tail -30 gpurun_out/r3l_encoder_attn.log; exit 1; }
cat gpurun_out/r3l_encoder_attn.jsonl
B="python scripts/bench_bert.py --steps 40 --warmup 10"
for seq in 128 512; do
  bs=64; [ $seq = 512 ] && bs=16
  for v in off on cu32 cu64 off; do
    ov=on; cus=0
    [ $v = off ] && ov=off
    [ $v = cu32 ] && cus=32
    [ $v = cu64 ] && cus=64
    DSA_OVERLAP_CUS=$cus timeout -k 10 200 $B --seq $seq --batch $bs --overlap-step $ov > gpurun_out/r3l_${seq}_$v.json 2> gpurun_out/r3l_${seq}_$v.log || { tail -30 gpurun_out/r3l_${seq}_$v.log; exit 1; }
    echo "$seq $v $(grep -o '"value": [0-9.]*' gpurun_out/r3l_${seq}_$v.json)"
  done
done
