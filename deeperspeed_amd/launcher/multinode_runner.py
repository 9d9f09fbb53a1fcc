"""Multi-node launch back-ends (reference parity: deepspeed/launcher/multinode_runner.py:1-292):
PDSH, OpenMPI, MVAPICH, Slurm and MosaicML.  Each builds the command that starts
`deeperspeed_amd.launcher.launch` (PDSH) or the user script directly (MPI/Slurm, rank from the
MPI environment) on every node."""

import json
import os
import shutil
import sys
from abc import ABC, abstractmethod
from shlex import quote

from .constants import MVAPICH_TMP_HOSTFILE, PDSH_MAX_FAN_OUT


class MultiNodeRunner(ABC):
    def __init__(self, args, world_info_base64):
        self.args = args
        self.user_arguments = self.parse_user_args()
        self.user_script = args.user_script
        self.world_info_base64 = world_info_base64
        self.exports = {}

    @abstractmethod
    def backend_exists(self):
        ...

    @abstractmethod
    def get_cmd(self, environment, active_resources):
        ...

    def add_export(self, key, var):
        self.exports[key.strip()] = var.strip()

    def parse_user_args(self):
        return self.args.user_args

    @property
    def name(self):
        return self.__class__.__name__


class PDSHRunner(MultiNodeRunner):
    def backend_exists(self):
        return shutil.which("pdsh") is not None

    def parse_user_args(self):
        return [x if x.startswith("-") else f"'{x}'" for x in self.args.user_args]

    def get_cmd(self, environment, active_resources):
        environment["PDSH_RCMD_TYPE"] = "ssh"
        active_workers = ",".join(active_resources.keys())
        pdsh_cmd_args = ["pdsh", "-f", str(PDSH_MAX_FAN_OUT), "-w", active_workers]
        if self.args.launcher_args:
            pdsh_cmd_args += self.args.launcher_args.split()
        exports = "".join(f"export {k}={quote(v)}; " for k, v in self.exports.items())
        launch = [exports + f"cd {os.path.abspath('.')};", sys.executable, "-u", "-m",
                  "deeperspeed_amd.launcher.launch", f"--world_info={self.world_info_base64}", "--node_rank=%n",
                  f"--master_addr={self.args.master_addr}", f"--master_port={self.args.master_port}"]
        return pdsh_cmd_args + launch + [self.user_script] + self.user_arguments


class OpenMPIRunner(MultiNodeRunner):
    def __init__(self, args, world_info_base64, resource_pool):
        super().__init__(args, world_info_base64)
        self.resource_pool = resource_pool
        self.add_export("UCX_TLS", "tcp")

    def backend_exists(self):
        return shutil.which("ompi_info") is not None

    def get_cmd(self, environment, active_resources):
        if self.args.include != "" or self.args.exclude != "" or self.args.num_nodes > 0 or self.args.num_gpus > 0:
            raise ValueError(f"{self.name} backend does not support worker include/exclusion/num_nodes/num_gpus")
        total = sum(self.resource_pool.values())
        cmd = ["mpirun", "-n", str(total), "-hostfile", self.args.hostfile, "--mca", "btl", "^openib", "--mca",
               "btl_tcp_if_include", "eth0"]
        if self.args.launcher_args:
            cmd += self.args.launcher_args.split()
        for k, v in self.exports.items():
            cmd += ["-x", f"{k}={quote(v)}"]
        return cmd + [sys.executable, "-u", self.user_script] + self.user_arguments


class MVAPICHRunner(MultiNodeRunner):
    def __init__(self, args, world_info_base64, resource_pool):
        super().__init__(args, world_info_base64)
        self.resource_pool = resource_pool
        self.add_export("MV2_SMP_USE_CMA", "0")
        self.add_export("MV2_DEBUG_SHOW_BACKTRACE", "1")
        self.add_export("MV2_SUPPORT_DL", "1")
        self.add_export("MV2_USE_ALIGNED_ALLOC", "1")

    def backend_exists(self):
        return shutil.which("mpiname") is not None

    def get_cmd(self, environment, active_resources):
        if self.args.include != "" or self.args.exclude != "" or self.args.num_nodes > 0 or self.args.num_gpus > 0:
            raise ValueError(f"{self.name} backend does not support worker include/exclusion/num_nodes/num_gpus")
        devices = list(self.resource_pool.values())
        if len(set(devices)) != 1:
            raise ValueError("mvapich requires the same number of devices per node")
        with open(MVAPICH_TMP_HOSTFILE, "w") as f:
            for host in self.resource_pool:
                f.write(f"{host}\n")
        cmd = ["mpirun", "-np", str(sum(devices)), "-ppn", str(devices[0]), "--hostfile", MVAPICH_TMP_HOSTFILE]
        if self.args.launcher_args:
            cmd += self.args.launcher_args.split()
        for k, v in self.exports.items():
            cmd += ["-env", f"{k}={quote(v)}"]
        return cmd + [sys.executable, "-u", self.user_script] + self.user_arguments


class SlurmRunner(MultiNodeRunner):
    def __init__(self, args, world_info_base64, resource_pool):
        super().__init__(args, world_info_base64)
        self.resource_pool = resource_pool

    def backend_exists(self):
        return shutil.which("sinfo") is not None

    def get_cmd(self, environment, active_resources):
        total = sum(self.resource_pool.values())
        cmd = ["srun", "-n", str(total)]
        if self.args.comment:
            cmd += ["--comment", self.args.comment]
        if self.args.include:
            cmd += ["--nodelist", self.args.include]
        if self.args.exclude:
            cmd += ["--exclude", self.args.exclude]
        if self.args.num_nodes > 0:
            cmd += ["--nodes", str(self.args.num_nodes)]
        if self.args.num_gpus > 0:
            cmd += ["--gpus", str(self.args.num_gpus)]
        if self.args.launcher_args:
            cmd += self.args.launcher_args.split()
        exports = "--export=ALL" + "".join(f",{k}={v}" for k, v in self.exports.items())
        return cmd + [exports, sys.executable, "-u", self.user_script] + self.user_arguments


class MosaicMLRunner(MultiNodeRunner):
    """MosaicML platform back-end (reference multinode_runner.py:256-292).  The platform starts
    one copy of this command per node and provides NODE_RANK / MASTER_ADDR / MASTER_PORT in the
    environment; JSON user arguments are re-serialised compactly (and nested `config_files`
    strings decoded) so they survive the platform's argument passing."""

    def backend_exists(self):
        return True

    def parse_user_args(self):
        out = []
        for arg in self.args.user_args:
            if arg.startswith("{") and arg.endswith("}"):
                try:
                    d = json.loads(arg)
                    if "config_files" in d:
                        d["config_files"] = {k: json.loads(v) for k, v in d["config_files"].items()}
                except json.JSONDecodeError as e:
                    raise ValueError("user arguments must be plain JSON (no comments, lowercase true/false)") from e
                arg = json.dumps(d, separators=(",", ":"))
            out.append(arg)
        return out

    def get_cmd(self, environment, active_resources):
        for key in ("NODE_RANK", "MASTER_ADDR", "MASTER_PORT"):
            if key not in os.environ:
                raise RuntimeError(f"{self.name}: {key} must be set by the platform")
        return [sys.executable, "-u", "-m", "deeperspeed_amd.launcher.launch", f"--world_info={self.world_info_base64}",
                f"--node_rank={os.environ['NODE_RANK']}", f"--master_addr={os.environ['MASTER_ADDR']}",
                f"--master_port={os.environ['MASTER_PORT']}", self.user_script] + self.user_arguments
