"""HBM <-> pinned-host copy rates on this box, alone and beside a bf16 GEMM stream: how much
PCIe slack a step has for parking activations (fc1 outputs) in host memory.  One JSON line per
case: GB/s of the copies and the GEMM's TF/s with and without them."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

MB = 1 << 20
n = 256 * MB // 2
dev = torch.device("cuda", 0)
x = torch.randn(n, device=dev).to(torch.bfloat16)
y = torch.empty_like(x)
h = torch.empty(n, dtype=torch.bfloat16, pin_memory=True)
h2 = torch.empty(n, dtype=torch.bfloat16, pin_memory=True)
h2.copy_(x.cpu())
a = torch.randn(8192, 6144, device=dev, dtype=torch.bfloat16)
w = torch.randn(24576, 6144, device=dev, dtype=torch.bfloat16)
s_d2h, s_h2d = torch.cuda.Stream(), torch.cuda.Stream()
REPS = 8


def gemm_loop(k):
    for _ in range(k):
        torch.nn.functional.linear(a, w)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.time()
    fn()
    torch.cuda.synchronize()
    return time.time() - t0


def d2h():
    with torch.cuda.stream(s_d2h):
        for _ in range(REPS):
            h.copy_(x, non_blocking=True)


def h2d():
    with torch.cuda.stream(s_h2d):
        for _ in range(REPS):
            y.copy_(h2, non_blocking=True)


gemm_loop(3)
d2h()
h2d()
gb = REPS * n * 2 / 1e9
flop = 2.0 * 8192 * 24576 * 6144
K = 40
t_g = timed(lambda: gemm_loop(K))
out = {"gemm_alone_tflops": round(K * flop / t_g / 1e12, 1)}
out["d2h_alone_gbps"] = round(gb / timed(d2h), 1)
out["h2d_alone_gbps"] = round(gb / timed(h2d), 1)
out["duplex_gbps_each"] = round(gb / timed(lambda: (d2h(), h2d())), 1)
t = timed(lambda: (d2h(), h2d(), gemm_loop(K)))
out["gemm_with_duplex_copies_tflops"] = round(K * flop / t / 1e12, 1)
out["copy_bytes_each_way_gb"] = gb
print(json.dumps(out), flush=True)
