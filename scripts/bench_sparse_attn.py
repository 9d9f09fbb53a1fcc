"""Attention fwd+bwd time at long sequence: dense causal flash vs block-sparse flash (fused
LUT walk) vs the unfused block-sparse path (SDD -> sparse softmax -> DSD), HIP events.

    python scripts/bench_sparse_attn.py --seq 8192 --heads 64 --dim 96 --mode bigbird --block 64
Prints one JSON line per variant (ms fwd+bwd, speed-up vs dense).  Reference claim: up to 6.3x
over dense (docs/_posts/2020-09-09-sparse-attention.md:33)."""
import argparse
import json
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--heads", type=int, default=64)
    ap.add_argument("--dim", type=int, default=96)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--mode", default="bigbird")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--unfused", action="store_true", help="also time the SDD/softmax/DSD path")
    ap.add_argument("--masked", action="store_true",
                    help="also time the fused kernels with a BERT-style key-padding mask (score bias)")
    a = ap.parse_args()
    from deeperspeed_amd.ops import native
    from deeperspeed_amd.ops.sparse_attention import sparsity_config as sc
    from deeperspeed_amd.ops.sparse_attention.flash import SparseFlashLUT, sparse_flash_attention
    from deeperspeed_amd.ops.sparse_attention.matmul import MatMul
    from deeperspeed_amd.ops.sparse_attention.softmax import Softmax
    random.seed(0)
    torch.manual_seed(0)
    B, H, S, D = a.batch, a.heads, a.seq, a.dim
    cls = {"bigbird": sc.BigBirdSparsityConfig, "fixed": sc.FixedSparsityConfig,
           "bslongformer": sc.BSLongformerSparsityConfig, "variable": sc.VariableSparsityConfig}[a.mode]
    cfg = cls(num_heads=H, block=a.block, attention="unidirectional")
    layout = cfg.make_layout(S)
    dev = torch.device("cuda")
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    g = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
    lut = SparseFlashLUT(layout, a.block, causal=True)

    def time_it(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    # autograd.grad, not backward(): accumulating into q/k/v.grad would add three elementwise
    # passes over [B, H, S, D] per call to the timed region
    def dense():
        o = native.flash_attention(q, k, v, True, D ** -0.5, out_layout="bshd")
        torch.autograd.grad(o, (q, k, v), g)

    def sparse():
        o = sparse_flash_attention(q, k, v, lut, D ** -0.5, out_bshd=True)
        torch.autograd.grad(o, (q, k, v), g)

    def sparse_fwd():
        with torch.no_grad():
            sparse_flash_attention(q, k, v, lut, D ** -0.5, out_bshd=True)

    def dense_fwd():
        with torch.no_grad():
            native.flash_attention(q, k, v, True, D ** -0.5, out_layout="bshd")

    flops_dense = 4 * B * H * S * S * D / 2 * 3.5  # causal, fwd + bwd(2.5x)
    t_dense = time_it(dense)
    t_sparse = time_it(sparse)
    t_dense_f, t_sparse_f = time_it(dense_fwd), time_it(sparse_fwd)
    res = [{"variant": "dense causal flash", "ms_fwd_bwd": round(t_dense, 3), "ms_fwd": round(t_dense_f, 3),
            "tflops": round(flops_dense / t_dense / 1e9, 1)},
           {"variant": f"block-sparse flash ({a.mode}, block {a.block})", "ms_fwd_bwd": round(t_sparse, 3),
            "ms_fwd": round(t_sparse_f, 3),
            "tile_density": round(lut.density, 4), "speedup_vs_dense": round(t_dense / t_sparse, 2),
            "effective_tflops": round(flops_dense * lut.density * 2 / t_sparse / 1e9, 1)}]
    if a.masked:
        from deeperspeed_amd.ops.sparse_attention.flash import score_biases
        kpm = torch.zeros(B, S, device=dev, dtype=torch.bfloat16)
        kpm[:, S - S // 8:] = -10000.0  # the last eighth of every sequence is padding
        kbias, _ = score_biases(q, key_padding_mask=kpm)

        def masked():
            o = sparse_flash_attention(q, k, v, lut, D ** -0.5, out_bshd=True, kbias=kbias)
            torch.autograd.grad(o, (q, k, v), g)
        t_m = time_it(masked)
        res.append({"variant": f"block-sparse flash ({a.mode}, block {a.block}) + key-padding mask",
                    "ms_fwd_bwd": round(t_m, 3), "vs_unmasked": round(t_m / t_sparse, 3),
                    "speedup_vs_dense": round(t_dense / t_m, 2)})
    if a.unfused:
        lay = layout.cpu()
        sdd, dsd, sm = MatMul(lay, a.block, "sdd", trans_b=True), MatMul(lay, a.block, "dsd"), Softmax(lay, a.block)

        def unfused():
            w = sm(sdd(q * D ** -0.5, k), scale=1.0, causal=True)
            o = dsd(w, v)
            torch.autograd.grad(o, (q, k, v), g.transpose(1, 2))
        t_u = time_it(unfused)
        res.append({"variant": "block-sparse SDD/softmax/DSD (unfused)", "ms_fwd_bwd": round(t_u, 3),
                    "speedup_vs_dense": round(t_dense / t_u, 2)})
    for r in res:
        r.update(B=B, H=H, S=S, D=D)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
