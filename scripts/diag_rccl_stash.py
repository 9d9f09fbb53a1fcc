"""How long does ProcessGroupNCCL (RCCL) keep references to an async collective's tensors?
Prints the storage use count of the output after wait(), after dropping the work and after
the watchdog has had time to observe completion.  Diagnostic only."""
import os
import time

import torch
import torch.distributed as dist

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29623"), RANK="0",
                  WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl")


def uc(t):
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata)


x = torch.randn(1 << 20, device="cuda", dtype=torch.bfloat16)
out = torch.empty_like(x)
w = dist.all_gather_into_tensor(out, x, async_op=True)
print("AVOID_RECORD_STREAMS", os.environ.get("TORCH_NCCL_AVOID_RECORD_STREAMS"), "before wait", uc(out))
w.wait()
print("after wait", uc(out))
del w
print("after del work", uc(out))
torch.cuda.synchronize()
time.sleep(1.0)
print("after 1s", uc(out))
dist.destroy_process_group()
