"""Per-node process launcher (reference parity: deepspeed/launcher/launch.py:1-179).

Starts one training process per selected MI355X with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set and HIP_VISIBLE_DEVICES restricted to this node's slots,
forwards SIGINT/SIGTERM to every child, and tears the whole node down as soon as one rank
fails (exit code of the first failure is returned).  Children are started with
`subprocess.Popen` (never exec) so no process that touched the GPU is replaced.
"""

import base64
import json
import os
import signal
import subprocess
import sys
import time
from argparse import REMAINDER, ArgumentParser

from ..utils.logging import logger


def parse_args(args=None):
    p = ArgumentParser(description="deeperspeed_amd per-node launcher: spawns one process per GPU")
    p.add_argument("--node_rank", type=int, default=0, help="Rank of this node in the multi-node setup.")
    p.add_argument("--master_addr", default="127.0.0.1", type=str, help="Master node (rank 0) address.")
    p.add_argument("--master_port", default=29500, type=int, help="Master node free port.")
    p.add_argument("--world_info", default="None", type=str, help="base64 world info: {host: [slot ids]}.")
    p.add_argument("--detect_xgmi_pairs", "--detect_nvlink_pairs", dest="detect_xgmi_pairs", action="store_true",
                   help="Order HIP_VISIBLE_DEVICES by xGMI adjacency.")
    p.add_argument("--bind_numa", action="store_true", help="Bind each rank to its GPU's NUMA node (numactl).")
    p.add_argument("training_script", type=str, help="Training program followed by its arguments.")
    p.add_argument("training_script_args", nargs=REMAINDER)
    return p.parse_args(args=args)


def build_rank_env(world_info, node_rank, master_addr, master_port, base_env=None, device_order=None):
    """[(env, local_rank)] for this node's processes."""
    nodes = list(world_info.keys())
    local_node = nodes[node_rank]
    local_slots = world_info[local_node]
    if device_order:
        local_slots = [s for s in device_order if s in local_slots]
    global_rank_mapping, cur = {}, 0
    for node, slots in world_info.items():
        global_rank_mapping[node] = list(range(cur, cur + len(slots)))
        cur += len(slots)
    world_size = cur
    env = dict(base_env if base_env is not None else os.environ)
    env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, local_slots))
    env.pop("CUDA_VISIBLE_DEVICES", None)  # one visibility mask on ROCm
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MASTER_ADDR"] = master_addr
    env["MASTER_PORT"] = str(master_port)
    env["WORLD_SIZE"] = str(world_size)
    env["LOCAL_SIZE"] = str(len(local_slots))
    env["CROSS_RANK"] = str(node_rank)
    env["CROSS_SIZE"] = str(len(nodes))
    out = []
    for local_rank in range(len(local_slots)):
        e = dict(env)
        e["RANK"] = str(global_rank_mapping[local_node][local_rank])
        e["LOCAL_RANK"] = str(local_rank)
        out.append(e)
    return out


def main(args=None):
    args = parse_args(args)
    world_info = json.loads(base64.urlsafe_b64decode(args.world_info))
    device_order = None
    if args.detect_xgmi_pairs:
        from .gpu_topology import get_topology_matrix, get_visible_device_order
        topo = get_topology_matrix()
        if topo:
            device_order = get_visible_device_order(topo)
    envs = build_rank_env(world_info, args.node_rank, args.master_addr, args.master_port, os.environ, device_order)
    processes = []
    for e in envs:
        cmd = [sys.executable, "-u", args.training_script, f"--local_rank={e['LOCAL_RANK']}"] + \
            args.training_script_args
        if args.bind_numa:
            from .gpu_topology import gpu_numa_node
            slot = int(e["HIP_VISIBLE_DEVICES"].split(",")[int(e["LOCAL_RANK"])])
            node = gpu_numa_node(slot)
            if node >= 0:
                cmd = ["numactl", f"--cpunodebind={node}", f"--membind={node}"] + cmd
        processes.append(subprocess.Popen(cmd, env=e))
    logger.info(f"launched {len(processes)} processes on node {args.node_rank}")

    def sigkill_handler(signum, frame):
        for p in processes:
            if p.poll() is None:
                try:
                    p.terminate()
                except ProcessLookupError:
                    pass
        time.sleep(1)
        for p in processes:
            if p.poll() is None:
                p.kill()
        sys.exit(1 if signum is None else 128 + int(signum))

    signal.signal(signal.SIGINT, sigkill_handler)
    signal.signal(signal.SIGTERM, sigkill_handler)
    alive = set(processes)
    while alive:
        finished = set()
        for p in alive:
            rc = p.poll()
            if rc is None:
                continue
            finished.add(p)
            if rc != 0:
                logger.error(f"process {p.pid} exited with code {rc}; terminating the node")
                for q in processes:
                    if q.poll() is None:
                        q.terminate()
                for q in processes:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                sys.exit(rc)
        alive -= finished
        time.sleep(0.2)


if __name__ == "__main__":
    main()
