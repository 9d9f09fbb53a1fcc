"""GPU interconnect topology for the launcher (reference: launcher/gpu_topology.py, which
pairs NVLink-bridged GPUs).  On MI355X every GPU of a node has a direct xGMI link to every
other one, so the useful information is (a) which GPUs are xGMI peers (to order
HIP_VISIBLE_DEVICES so adjacent ranks are direct peers on partially connected systems) and
(b) each GPU's NUMA node (to bind each rank's CPU threads next to its GPU)."""

import json
import os
import re
import subprocess
from typing import Dict, List, Optional, Set, Tuple


def get_topology_matrix() -> Optional[List[List[str]]]:
    """Link-type matrix from `rocm-smi --showtopotype --json` ("XGMI" / "PCIE"), or None."""
    try:
        out = subprocess.check_output(["rocm-smi", "--showtopotype", "--json"], stderr=subprocess.DEVNULL,
                                      timeout=20).decode()
        data = json.loads(out)
    except Exception:
        return None
    links: Dict[Tuple[int, int], str] = {}
    n = 0
    for _, entries in data.items():
        for key, val in entries.items():
            m = re.search(r"GPU (\d+) to GPU (\d+)", key)
            if m:
                a, b = int(m.group(1)), int(m.group(2))
                links[(a, b)] = str(val)
                n = max(n, a + 1, b + 1)
    if n == 0:
        return None
    return [["X" if i == j else links.get((i, j), links.get((j, i), "PCIE")) for j in range(n)] for i in range(n)]


def is_xgmi(link: str) -> bool:
    return "XGMI" in link.upper()


def get_xgmi_pairs(topology) -> Set[Tuple[int, int]]:
    out = set()
    for i, row in enumerate(topology):
        for j, link in enumerate(row):
            if i < j and is_xgmi(link):
                out.add((i, j))
    return out


def get_visible_device_order(topology=None, local_gpu_ids: Optional[List[int]] = None) -> List[int]:
    """Order GPUs so consecutive local ranks are xGMI peers where possible."""
    ids = list(local_gpu_ids) if local_gpu_ids is not None else list(range(len(topology or [])))
    if not topology:
        return ids
    order, left = [ids[0]], set(ids[1:])
    while left:
        cur = order[-1]
        peers = sorted(g for g in left if is_xgmi(topology[cur][g]))
        nxt = peers[0] if peers else min(left)
        order.append(nxt)
        left.remove(nxt)
    return order


def gpu_numa_node(gpu_index: int) -> int:
    """NUMA node of a GPU from sysfs (-1 when unknown)."""
    drm = "/sys/class/drm"
    try:
        cards = sorted(d for d in os.listdir(drm) if re.fullmatch(r"card\d+", d))
    except OSError:
        return -1
    gpus = []
    for c in cards:
        dev = os.path.join(drm, c, "device")
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip() != "0x1002":
                    continue
            with open(os.path.join(dev, "numa_node")) as f:
                gpus.append(int(f.read().strip()))
        except OSError:
            continue
    return gpus[gpu_index] if gpu_index < len(gpus) else -1
