"""Probe: can two RCCL ranks share one GPU on this box?  Each rank runs the collectives the
engine uses (all_reduce, reduce_scatter_tensor, all_gather_into_tensor, all_to_all_single,
batched isend/irecv) on cuda:0 and checks the results.  Prints one JSON line per rank.

    python scripts/rccl_two_ranks_one_gpu.py [--world 2]
"""

import argparse
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    res = {"rank": rank}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        dev = torch.device("cuda", 0)
        n = 1 << 20
        x = torch.full((n,), float(rank + 1), device=dev, dtype=torch.bfloat16)
        dist.all_reduce(x)
        res["all_reduce"] = float(x[0]) == world * (world + 1) / 2
        big = torch.arange(world * n, device=dev, dtype=torch.float32) + rank
        out = torch.empty(n, device=dev)
        dist.reduce_scatter_tensor(out, big)
        ref = (torch.arange(world * n, device=dev, dtype=torch.float32) * world + world * (world - 1) / 2)[rank * n:(rank + 1) * n]
        res["reduce_scatter"] = bool(torch.equal(out, ref))
        shard = torch.full((n,), float(rank), device=dev)
        full = torch.empty(world * n, device=dev)
        dist.all_gather_into_tensor(full, shard)
        res["all_gather"] = bool(all(float(full[r * n]) == r for r in range(world)))
        a = torch.arange(world * 4, device=dev, dtype=torch.float32) + 100 * rank
        b = torch.empty_like(a)
        dist.all_to_all_single(b, a)
        res["all_to_all"] = bool(all(float(b[4 * r]) == 100 * r + 4 * rank for r in range(world)))
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        s = torch.full((1024,), float(rank), device=dev)
        r_ = torch.empty(1024, device=dev)
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, s, nxt), dist.P2POp(dist.irecv, r_, prv)])
        for w in reqs:
            w.wait()
        res["p2p"] = float(r_[0]) == float(prv)
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
        res["ok"] = all(v for k, v in res.items() if k != "rank")
    except Exception as e:  # noqa: BLE001
        res["ok"] = False
        res["error"] = repr(e)[:400]
    q.put(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    out = []
    for _ in ps:
        out.append(q.get(timeout=180))
    for p in ps:
        p.join(timeout=30)
    for r in sorted(out, key=lambda d: d["rank"]):
        print(json.dumps(r), flush=True)
    sys.exit(0 if all(r.get("ok") for r in out) else 1)


if __name__ == "__main__":
    main()
