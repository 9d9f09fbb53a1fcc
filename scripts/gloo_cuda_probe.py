"""gloo collectives on GPU tensors (N ranks sharing one GPU, the one-GPU rehearsal of an N-GPU
job): time reduce_scatter_tensor / all_gather_into_tensor / all_reduce per dtype and size, to
tell gloo's throughput from a collective-order problem.  torchrun --nproc-per-node N."""
import json
import os
import time

import torch
import torch.distributed as dist

dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(0)
for n in (4_000_000, 26_000_000, 103_284_736):
    for dt in (torch.bfloat16, torch.float32):
        x = torch.ones(n - n % w, dtype=dt, device="cuda")
        out = torch.empty(x.numel() // w, dtype=dt, device="cuda")
        res = {}
        for name, fn in (("reduce_scatter", lambda: dist.reduce_scatter_tensor(out, x)),
                         ("all_gather", lambda: dist.all_gather_into_tensor(x, out)),
                         ("all_reduce", lambda: dist.all_reduce(x))):
            dist.barrier()
            torch.cuda.synchronize()
            t = time.time()
            fn()
            torch.cuda.synchronize()
            dist.barrier()
            res[name] = round(time.time() - t, 3)
        if r == 0:
            print(json.dumps({"world": w, "numel": n, "dtype": str(dt), "seconds": res}), flush=True)
dist.destroy_process_group()
