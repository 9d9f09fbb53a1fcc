"""Which hipMemcpy path a 64 MB HBM -> pinned-host copy takes (run under rocprofv3 --kernel-trace
--memory-copy-trace: copyBuffer kernels = blit copies on the CUs, memory-copy records = DMA engine)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from deeperspeed_amd.ops import native  # noqa: E402

n = 16 * 1024 * 1024
x = torch.randn(n, device="cuda")
h = torch.empty(n, dtype=torch.float32, pin_memory=True)
s = torch.cuda.Stream()
variants = {"torch_copy": lambda: h.copy_(x, non_blocking=True),
            "nocu": lambda: native.copy_nocu_(h, x),
            "kind_d2h": lambda: native.copy_nocu_(h, x, 2),
            "kind_default": lambda: native.copy_nocu_(h, x, 4),
            "narrow8": lambda: native.copy_narrow_(h, x, 8),
            "narrow16": lambda: native.copy_narrow_(h, x, 16),
            "narrow32": lambda: native.copy_narrow_(h, x, 32),
            "narrow64": lambda: native.copy_narrow_(h, x, 64)}
for name, fn in variants.items():
    with torch.cuda.stream(s):
        fn()
    s.synchronize()
    torch.cuda.synchronize()
    t0 = time.time()
    with torch.cuda.stream(s):
        for _ in range(10):
            fn()
    s.synchronize()
    dt = (time.time() - t0) / 10
    assert torch.equal(h, x.cpu()), name
    h.zero_()
    print(f"{name}: {dt * 1e3:.2f} ms per 64 MB copy ({64 / 1024 / dt:.1f} GB/s)", flush=True)
    time.sleep(0.05)
