"""`deepspeed`-style launcher front end (reference parity: deepspeed/launcher/runner.py:1-386).

    deepspeed [-H hostfile] [-i include] [-e exclude] [--num_nodes N] [--num_gpus G]
              [--master_addr A] [--master_port P] [--launcher pdsh|openmpi|mvapich|slurm]
              user_script.py user args...

Single node: starts `deeperspeed_amd.launcher.launch` locally (one process per MI355X).
Multi node: hands the per-node launch to PDSH / MPI / Slurm with the ROCm/RCCL environment
exported (NCCL_*, RCCL_*, HSA_*, HIP_*, ... plus `.deepspeed_env` files).
"""

import argparse
import base64
import collections
import json
import os
import subprocess
import sys
from copy import deepcopy

from ..utils.logging import logger
from .constants import (DEEPSPEED_ENVIRONMENT_NAME, DEFAULT_HOSTFILE, EXPORT_ENVS, MOSAICML_LAUNCHER, MVAPICH_LAUNCHER,
                        OPENMPI_LAUNCHER, PDSH_LAUNCHER, SLURM_LAUNCHER, TORCH_DISTRIBUTED_DEFAULT_PORT)

DEEPSPEED_ENVIRONMENT_PATHS = [os.path.expanduser("~"), "."]


def parse_args(args=None):
    p = argparse.ArgumentParser(description="deeperspeed_amd runner: launch distributed multi-node/multi-GPU "
                                            "training jobs on MI355X.")
    p.add_argument("-H", "--hostfile", type=str, default=DEFAULT_HOSTFILE,
                   help="Hostfile path (MPI style: `hostname slots=N`).")
    p.add_argument("-i", "--include", type=str, default="",
                   help="Resources to use, e.g. `worker-0@worker-1:0,2` (mutually exclusive with --exclude).")
    p.add_argument("-e", "--exclude", type=str, default="",
                   help="Resources NOT to use, e.g. `worker-1:0`.")
    p.add_argument("--num_nodes", type=int, default=-1, help="Number of worker nodes to run on.")
    p.add_argument("--num_gpus", type=int, default=-1, help="Max number of GPUs to use on each node.")
    p.add_argument("--master_port", default=TORCH_DISTRIBUTED_DEFAULT_PORT, type=int,
                   help="Port used by torch.distributed for communication during training.")
    p.add_argument("--master_addr", default="", type=str, help="IP address of node 0.")
    p.add_argument("--launcher", default=PDSH_LAUNCHER, type=str,
                   help="Multi-node launcher backend: pdsh, openmpi, mvapich, slurm, mosaicml.")
    p.add_argument("--launcher_args", default="", type=str, help="Extra arguments for the launcher backend.")
    p.add_argument("--force_multi", action="store_true", help="Force multi-node launch mode on one node.")
    p.add_argument("--comment", default="", type=str, help="Slurm --comment.")
    p.add_argument("--detect_xgmi_pairs", "--detect_nvlink_pairs", dest="detect_xgmi_pairs", action="store_true",
                   help="Order HIP_VISIBLE_DEVICES so consecutive ranks are xGMI peers.")
    p.add_argument("user_script", type=str, help="User script to launch, followed by its arguments.")
    p.add_argument("user_args", nargs=argparse.REMAINDER)
    return p.parse_args(args=args)


def fetch_hostfile(hostfile_path):
    if not os.path.isfile(hostfile_path):
        logger.warning("Unable to find hostfile, will proceed with training with local resources only.")
        return None
    resource_pool = collections.OrderedDict()
    with open(hostfile_path) as fd:
        for line in fd.readlines():
            line = line.strip()
            if line == "" or line.startswith("#"):
                continue
            try:
                hostname, slots = line.split()
                _, slot_count = slots.split("=")
                slot_count = int(slot_count)
            except ValueError as err:
                logger.error("Hostfile is not formatted correctly, unable to proceed with training.")
                raise err
            if hostname in resource_pool:
                logger.error("Hostfile contains duplicate hosts, unable to proceed with training.")
                raise ValueError(f"host {hostname} is already defined")
            resource_pool[hostname] = slot_count
    return resource_pool


def _parse_filter(s):
    """`host1:0,2@host2` -> {host1: [0, 2], host2: []} (empty list = all slots)."""
    out = collections.OrderedDict()
    for node in s.split("@"):
        if not node:
            continue
        if ":" in node:
            host, slots = node.split(":")
            out[host] = [int(x) for x in slots.split(",")]
        else:
            out[node] = []
    return out


def parse_resource_filter(host_info, include_str="", exclude_str=""):
    """Apply --include/--exclude to {host: [slot ids]} (reference runner.py:160-250)."""
    if include_str and exclude_str:
        raise ValueError("include_str and exclude_str are mutually exclusive.")
    if not include_str and not exclude_str:
        return host_info
    filtered = collections.OrderedDict()
    if include_str:
        for host, slots in _parse_filter(include_str).items():
            if host not in host_info:
                raise ValueError(f"Hostname '{host}' not found in hostfile")
            for s in slots:
                if s not in host_info[host]:
                    raise ValueError(f"No slot '{s}' specified on host '{host}'")
            filtered[host] = slots if slots else list(host_info[host])
        return filtered
    excl = _parse_filter(exclude_str)
    for host, slots in host_info.items():
        if host in excl:
            if not excl[host]:
                continue  # whole host excluded
            for s in excl[host]:
                if s not in slots:
                    raise ValueError(f"No slot '{s}' specified on host '{host}'")
            keep = [s for s in slots if s not in excl[host]]
            if keep:
                filtered[host] = keep
        else:
            filtered[host] = list(slots)
    for host in excl:
        if host not in host_info:
            raise ValueError(f"Hostname '{host}' not found in hostfile")
    return filtered


def parse_inclusion_exclusion(resource_pool, inclusion, exclusion):
    active = collections.OrderedDict((h, list(range(n))) for h, n in resource_pool.items())
    return parse_resource_filter(active, include_str=inclusion, exclude_str=exclusion)


def encode_world_info(world_info):
    return base64.urlsafe_b64encode(json.dumps(world_info).encode("utf-8")).decode("utf-8")


def decode_world_info(s):
    return json.loads(base64.urlsafe_b64decode(s))


def _local_gpu_count():
    try:
        import torch
        return torch.cuda.device_count()  # counting devices does not initialise HIP
    except Exception:
        return 0


def main(args=None):
    args = parse_args(args)
    resource_pool = fetch_hostfile(args.hostfile)
    if not resource_pool:
        resource_pool = collections.OrderedDict()
        n = _local_gpu_count()
        if n == 0 and args.num_gpus <= 0:
            raise RuntimeError("Unable to proceed, no GPU resources available")
        resource_pool["localhost"] = n if n > 0 else args.num_gpus
        args.master_addr = args.master_addr or "127.0.0.1"
        multi_node_exec = False
    else:
        multi_node_exec = len(resource_pool) > 1
    if not multi_node_exec and args.num_nodes > 1:
        raise ValueError("Num nodes is >1 but no extra nodes available via hostfile")
    active = parse_inclusion_exclusion(resource_pool, args.include, args.exclude)
    env = os.environ.copy()
    if not args.master_addr:
        first = list(active.keys())[0]
        hostname_cmd = [f"ssh {first} hostname -I"]
        result = subprocess.check_output(hostname_cmd, shell=True)
        args.master_addr = result.decode("utf-8").split()[0]
        logger.info(f"Using IP address of {args.master_addr} for node {first}")
    if args.num_nodes > 0:
        active = collections.OrderedDict(list(active.items())[:args.num_nodes])
    if args.num_gpus > 0:
        active = collections.OrderedDict((h, s[:args.num_gpus]) for h, s in active.items())
    world_info_base64 = encode_world_info(active)
    multi_node_exec = args.force_multi or len(active) > 1
    if not multi_node_exec:
        cmd = [sys.executable, "-u", "-m", "deeperspeed_amd.launcher.launch", f"--world_info={world_info_base64}",
               f"--master_addr={args.master_addr}", f"--master_port={args.master_port}"]
        if args.detect_xgmi_pairs:
            cmd.append("--detect_xgmi_pairs")
        cmd += [args.user_script] + args.user_args
    else:
        from .multinode_runner import MosaicMLRunner, MVAPICHRunner, OpenMPIRunner, PDSHRunner, SlurmRunner
        launcher = args.launcher.lower()
        if launcher == PDSH_LAUNCHER:
            runner = PDSHRunner(args, world_info_base64)
        elif launcher == OPENMPI_LAUNCHER:
            runner = OpenMPIRunner(args, world_info_base64, resource_pool)
        elif launcher == MVAPICH_LAUNCHER:
            runner = MVAPICHRunner(args, world_info_base64, resource_pool)
        elif launcher == SLURM_LAUNCHER:
            runner = SlurmRunner(args, world_info_base64, resource_pool)
        elif launcher == MOSAICML_LAUNCHER:
            runner = MosaicMLRunner(args, world_info_base64)
        else:
            raise NotImplementedError(f"Unknown launcher {args.launcher}")
        if not runner.backend_exists():
            raise RuntimeError(f"launcher '{args.launcher}' not installed.")
        curr_path = os.path.abspath(".")
        env["PYTHONPATH"] = curr_path + (":" + env["PYTHONPATH"] if "PYTHONPATH" in env else "")
        for var in env:
            if any(var.startswith(name) for name in EXPORT_ENVS):
                runner.add_export(var, env[var])
        for environ_path in DEEPSPEED_ENVIRONMENT_PATHS:
            environ_file = os.path.join(environ_path, DEEPSPEED_ENVIRONMENT_NAME)
            if os.path.isfile(environ_file):
                with open(environ_file) as fd:
                    for var in fd.readlines():
                        if "=" in var:
                            key, val = var.split("=", 1)
                            runner.add_export(key, val)
        cmd = runner.get_cmd(env, active)
    logger.info(f"cmd = {' '.join(cmd)}")
    result = subprocess.Popen(cmd, env=env)
    result.wait()
    if result.returncode > 0:
        sys.exit(result.returncode)


if __name__ == "__main__":
    main()
