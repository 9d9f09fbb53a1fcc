"""Rotary split kernels (QKV projection output -> rotated, scaled q / k / v and back) at the
GPT-NeoX-20B shape: time and HBM rate of each direction.

    python scripts/bench_rotary.py [--batch 4 --seq 2048 --heads 64 --hd 96 --rot 24]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deeperspeed_amd.ops import native  # noqa: E402
from deeperspeed_amd.ops.attention import rotary_table  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--heads", type=int, default=64)
    ap.add_argument("--hd", type=int, default=96)
    ap.add_argument("--rot", type=int, default=24)
    args = ap.parse_args()
    ops = native.hip_ops()
    B, S, NH, HD, R = args.batch, args.seq, args.heads, args.hd, args.rot
    qkv = torch.randn(B, S, NH * 3 * HD, device="cuda", dtype=torch.bfloat16)
    cs = rotary_table(S, R, 10000.0, qkv.device)
    dq, dk, dv = (torch.randn(B, NH, S, HD, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    nbytes = qkv.numel() * 2 * 2  # read + write of the QKV projection output
    tf = timed(lambda: ops.rotary_split_fwd(qkv, cs, NH, HD, R, 0.5))
    tb = timed(lambda: ops.rotary_split_bwd(dq, dk, dv, cs, R, 0.5))
    print(json.dumps({"B": B, "S": S, "NH": NH, "HD": HD, "rot": R, "fwd_us": round(tf * 1e3, 1),
                      "fwd_TBps": round(nbytes / tf / 1e9, 2), "bwd_us": round(tb * 1e3, 1),
                      "bwd_TBps": round(nbytes / tb / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
