"""rotary_split fwd/bwd at the GPT-NeoX-20B shape (B4 S2048 64 heads x 96, rotary 24):
achieved HBM bandwidth of the HIP kernels (bytes = read + write of q, k, v)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from deeperspeed_amd.ops import attention as A
    B, S, NH, HD, ROT = 4, 2048, 64, 96, 24
    dev = torch.device("cuda", 0)
    qkv = torch.randn(B, S, NH * 3 * HD, device=dev, dtype=torch.bfloat16)
    cs = A.rotary_table(S, ROT, 10000.0, dev)
    from deeperspeed_amd.ops import native
    ops = native.hip_ops()
    q, k, v = ops.rotary_split_fwd(qkv, cs, NH, HD, ROT, 0.1)
    nbytes = 2 * qkv.numel() * 2
    for name, fn in (("fwd", lambda: ops.rotary_split_fwd(qkv, cs, NH, HD, ROT, 0.1)),
                     ("bwd", lambda: ops.rotary_split_bwd(q, k, v, cs, ROT, 0.1))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 50
        print(json.dumps({"op": f"rotary_split_{name}", "us": round(ms * 1e3, 1), "TB/s": round(nbytes / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
