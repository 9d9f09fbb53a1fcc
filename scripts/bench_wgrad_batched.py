"""Weight gradients of BERT-Large's four linears: per layer (split-K over tokens, the per-layer path)
vs all 24 layers in one strided-batched GEMM (ops/wgrad_batch.py).  The round-5 probes of hipBLASLt's
grouped GEMM (every solution rejected with an internal error) and rocBLAS's pointer-array batched GEMM
(~3 TF/s) are recorded in profiles/r5f_wgrad_batched.jsonl."""
import json
import time

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.time() - t) / iters


def main():
    dev = torch.device("cuda")
    M, L = 8192, 24
    shapes = {"qkv": (3072, 1024), "attn_out": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096)}
    for name, (N, K) in shapes.items():
        dy = torch.randn(L, M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(L, M, K, device=dev, dtype=torch.bfloat16)
        gw = torch.zeros(L, N, K, device=dev, dtype=torch.bfloat16)
        flops = 2 * L * M * N * K

        def per_layer():
            for l in range(L):
                part = torch.bmm(dy[l].view(4, M // 4, N).transpose(1, 2), x[l].view(4, M // 4, K),
                                 out_dtype=torch.float32)
                gw[l].add_(part.sum(0).to(torch.bfloat16))

        def batched_nt():  # dW[l] += dy[l]^T x[l], token-major operands
            gw.baddbmm_(dy.transpose(1, 2), x)

        def batched_fp32():
            torch.bmm(dy.transpose(1, 2), x, out_dtype=torch.float32)

        r = {"linear": name, "N": N, "K": K, "M": M, "layers": L}
        for k, fn in (("per_layer_split4_ms", per_layer), ("batched_nt_ms", batched_nt), ("batched_f32out_ms", batched_fp32)):
            t = timeit(fn)
            r[k] = round(t * 1e3, 3)
            r[k.replace("_ms", "_tflops")] = round(flops / t / 1e12, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
