"""Rotary + QKV split fwd/bwd at the GPT-NeoX-20B shape (B4 S2048 NH64 HD96 rotary 24): the
LDS-tiled kernels vs the row-per-thread kernels (DSA_ROTARY_TILED=0), HIP events, one JSON line
per variant with the achieved HBM bandwidth (read + write of the full QKV tensor)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    from deeperspeed_amd.ops import attention as A
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4,2048,64,96,24", help="B,S,NH,HD,ROT (1.3B at 16x1: 16,2048,16,128,32)")
    B, S, NH, HD, ROT = (int(x) for x in ap.parse_args().shape.split(","))
    qkv = torch.randn(B, S, 3 * NH * HD, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    nbytes = 2 * qkv.numel() * 2

    def run(tiled):
        os.environ["DSA_ROTARY_TILED"] = str(int(tiled))
        q, k, v = A.rotary_split(qkv, NH, HD, ROT, qscale=HD ** -0.5)
        g = [torch.randn_like(t) for t in (q, k, v)]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for _ in range(3):
            A.rotary_split(qkv, NH, HD, ROT, qscale=HD ** -0.5)
        torch.cuda.synchronize()
        e[0].record()
        for _ in range(20):
            out = A.rotary_split(qkv, NH, HD, ROT, qscale=HD ** -0.5)
        e[1].record()
        e[2].record()
        for _ in range(20):
            torch.autograd.grad(out, qkv, g, retain_graph=True)
        e[3].record()
        torch.cuda.synchronize()
        fwd, fb = e[0].elapsed_time(e[1]) / 20, e[2].elapsed_time(e[3]) / 20
        return out, fwd, fb

    res = {}
    names = {0: "row-per-thread", 1: "tiled (padded LDS rows)", 2: "tiled (unpadded rows)"}
    for tiled in (0, 2, 1, 2, 1):
        out, fwd, bwd = run(tiled)
        res[tiled] = out
        print(json.dumps({"variant": names[tiled], "shape": [B, S, NH, HD, ROT], "fwd_us": round(fwd * 1e3, 1),
                          "bwd_us": round(bwd * 1e3, 1), "fwd_TBps": round(nbytes / fwd / 1e9, 2),
                          "bwd_TBps": round(nbytes / bwd / 1e9, 2)}), flush=True)
    assert all(torch.equal(a, b) for a, b in zip(res[0], res[1]))
    assert all(torch.equal(a, b) for a, b in zip(res[0], res[2]))


if __name__ == "__main__":
    main()
