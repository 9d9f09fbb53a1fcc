"""Probe: does a later BertForPreTraining instance in the same process run slower (r4aq saw the
third model at seq 512 take 39.1 ms vs 28.5 ms as the first)?  Times encode fwd+bwd for several
fresh instances in one process, with and without an HF BertModel built in between."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from deeperspeed_amd.models.bert import BertForPreTraining, get_config  # noqa: E402


def timed(m, ids, tt, am, iters=20, warmup=10):
    for _ in range(warmup):
        m.encode(ids, tt, am).float().sum().backward()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(iters):
        m.encode(ids, tt, am).float().sum().backward()
    torch.cuda.synchronize()
    return round((time.time() - t0) / iters * 1e3, 2)


dev = torch.device("cuda")
S, B = 512, 16
ids = torch.randint(0, 30528, (B, S), device=dev)
tt = torch.zeros(B, S, dtype=torch.long, device=dev)
am = torch.ones(B, S, dtype=torch.long, device=dev)
for i in range(4):
    m = BertForPreTraining(get_config("bert-large", max_position=512), device=dev, dtype=torch.bfloat16).train()
    print(json.dumps({"instance": i, "ms": timed(m, ids, tt, am),
                      "allocated_gib": round(torch.cuda.memory_allocated() / 2**30, 1)}), flush=True)
    del m
    torch.cuda.empty_cache()
