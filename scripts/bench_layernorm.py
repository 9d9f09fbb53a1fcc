"""LayerNorm (+ residual-gradient fusion) forward / backward at the GPT-NeoX 1.3B (16 x 2048 tokens,
hidden 2048) and 20B (4 x 2048 tokens, hidden 6144) shapes, HIP events, one JSON line per shape
with the achieved HBM bandwidth (fwd: read x + write y; bwd: read dy, x, dres + write dx)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from deeperspeed_amd.ops import native
    # the backward's row prefetch is chosen per hidden size in the launcher (norm_act.hip)
    for rows, H in ((32768, 2048), (8192, 6144), (32768, 2048), (8192, 6144)):
        x = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = torch.randn(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        b = torch.randn(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        dy = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16)
        dres = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16)
        y, xo = native.layer_norm_residual(x, w, b, 1e-5)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for _ in range(3):
            native.layer_norm_residual(x, w, b, 1e-5)
            torch.autograd.grad((y, xo), (x, w, b), (dy, dres), retain_graph=True)
        torch.cuda.synchronize()
        e[0].record()
        for _ in range(20):
            native.layer_norm_residual(x, w, b, 1e-5)
        e[1].record()
        e[2].record()
        for _ in range(20):
            torch.autograd.grad((y, xo), (x, w, b), (dy, dres), retain_graph=True)
        e[3].record()
        torch.cuda.synchronize()
        f, bw = e[0].elapsed_time(e[1]) / 20, e[2].elapsed_time(e[3]) / 20
        nb = rows * H * 2
        print(json.dumps({"rows": rows, "hidden": H, "fwd_us": round(f * 1e3, 1), "bwd_us": round(bw * 1e3, 1),
                          "fwd_TBps": round(2 * nb / f / 1e9, 2), "bwd_TBps": round(4 * nb / bw / 1e9, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
