"""Launcher (reference tests/unit/test_run.py): hostfile parsing, include/exclude filters,
world-info encoding, multinode command construction, and a real local 2-process launch
(gloo) including failure propagation."""

import base64
import json
import os
import subprocess
import sys
import textwrap
from types import SimpleNamespace

import pytest

from deeperspeed_amd.launcher import runner as dsrun
from deeperspeed_amd.launcher.launch import build_rank_env

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parser_mutual_exclusive():
    with pytest.raises(ValueError):
        dsrun.parse_resource_filter({}, include_str="A", exclude_str="B")


def test_parser_local():
    hosts = {"worker-0": [0, 1, 2, 3], "worker-1": [0, 1, 2, 3]}
    assert dsrun.parse_resource_filter(hosts) == hosts
    assert dsrun.parse_resource_filter(hosts, include_str="worker-0") == {"worker-0": [0, 1, 2, 3]}
    assert dsrun.parse_resource_filter(hosts, include_str="worker-1:0,3") == {"worker-1": [0, 3]}
    ret = dsrun.parse_resource_filter(hosts, include_str="worker-0:1@worker-1:0,3")
    assert ret == {"worker-0": [1], "worker-1": [0, 3]}
    ret = dsrun.parse_resource_filter(hosts, exclude_str="worker-1")
    assert ret == {"worker-0": [0, 1, 2, 3]}
    ret = dsrun.parse_resource_filter(hosts, exclude_str="worker-0:1@worker-1:0,3")
    assert ret == {"worker-0": [0, 2, 3], "worker-1": [1, 2]}
    with pytest.raises(ValueError):
        dsrun.parse_resource_filter(hosts, include_str="jeff")
    with pytest.raises(ValueError):
        dsrun.parse_resource_filter(hosts, include_str="worker-0:7")


def test_hostfile(tmp_path):
    hf = tmp_path / "hostfile"
    hf.write_text("# comment\nworker-0 slots=8\nworker-1 slots=4\n\n")
    pool = dsrun.fetch_hostfile(str(hf))
    assert list(pool.items()) == [("worker-0", 8), ("worker-1", 4)]
    hf.write_text("worker-0 slots=8\nworker-0 slots=8\n")
    with pytest.raises(ValueError):
        dsrun.fetch_hostfile(str(hf))
    assert dsrun.fetch_hostfile(str(tmp_path / "missing")) is None


def test_world_info_and_rank_env():
    wi = {"a": [0, 1], "b": [2, 3, 5]}
    enc = dsrun.encode_world_info(wi)
    assert dsrun.decode_world_info(enc) == wi
    envs = build_rank_env(wi, 1, "10.0.0.1", 1234, base_env={})
    assert [e["RANK"] for e in envs] == ["2", "3", "4"]
    assert all(e["WORLD_SIZE"] == "5" and e["HIP_VISIBLE_DEVICES"] == "2,3,5" for e in envs)
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]


def test_multinode_cmds():
    from deeperspeed_amd.launcher.multinode_runner import OpenMPIRunner, PDSHRunner, SlurmRunner
    args = SimpleNamespace(user_script="train.py", user_args=["--x", "1"], launcher_args="", master_addr="h0",
                           master_port=29500, include="", exclude="", num_nodes=-1, num_gpus=-1,
                           hostfile="/job/hostfile", comment="")
    wi = dsrun.encode_world_info({"h0": [0], "h1": [0]})
    pd = PDSHRunner(args, wi)
    pd.add_export("NCCL_DEBUG", "INFO")
    cmd = pd.get_cmd({}, {"h0": [0], "h1": [0]})
    assert cmd[:5] == ["pdsh", "-f", "1024", "-w", "h0,h1"] and "train.py" in cmd
    assert any("export NCCL_DEBUG=INFO" in c for c in cmd)
    args.num_nodes, args.num_gpus = 0, 0
    om = OpenMPIRunner(args, wi, {"h0": 8, "h1": 8})
    args.num_nodes = args.num_gpus = -1
    om.args.num_nodes = 0
    om.args.num_gpus = 0
    cmd = om.get_cmd({}, {})
    assert cmd[:3] == ["mpirun", "-n", "16"]
    sl = SlurmRunner(args, wi, {"h0": 8})
    assert sl.get_cmd({}, {})[:3] == ["srun", "-n", "8"]


def test_mosaicml_runner(monkeypatch):
    from deeperspeed_amd.launcher.multinode_runner import MosaicMLRunner
    args = SimpleNamespace(user_script="train.py", launcher_args="",
                           user_args=['{"a": true, "config_files": {"c": "{\\"x\\": 1}"}}', "--y"])
    wi = dsrun.encode_world_info({"h0": [0, 1]})
    mm = MosaicMLRunner(args, wi)
    assert mm.user_arguments == ['{"a":true,"config_files":{"c":{"x":1}}}', "--y"]
    monkeypatch.setenv("NODE_RANK", "3")
    monkeypatch.setenv("MASTER_ADDR", "10.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "1234")
    cmd = mm.get_cmd({}, {})
    assert cmd[2:4] == ["-m", "deeperspeed_amd.launcher.launch"]
    assert "--node_rank=3" in cmd and "--master_addr=10.0.0.1" in cmd and cmd[-3:] == ["train.py"] + mm.user_arguments
    with pytest.raises(ValueError):
        MosaicMLRunner(SimpleNamespace(user_script="t.py", user_args=["{bad}"]), wi)


_SCRIPT = textwrap.dedent("""
    import os, sys, argparse
    import torch.distributed as dist
    p = argparse.ArgumentParser(); p.add_argument("--local_rank", type=int); p.add_argument("--fail", type=int, default=-1)
    a = p.parse_args()
    assert int(os.environ["LOCAL_RANK"]) == a.local_rank
    if int(os.environ["RANK"]) == a.fail:
        sys.exit(3)
    dist.init_process_group("gloo")
    import torch
    t = torch.ones(1) * (dist.get_rank() + 1)
    dist.all_reduce(t)
    assert t.item() == 3.0
    dist.destroy_process_group()
""")


def _launch(tmp_path, extra):
    script = tmp_path / "train.py"
    script.write_text(_SCRIPT)
    wi = dsrun.encode_world_info({"localhost": [0, 1]})
    env = dict(os.environ, PYTHONPATH=REPO)
    port = 29600 + os.getpid() % 300
    return subprocess.run([sys.executable, "-m", "deeperspeed_amd.launcher.launch", f"--world_info={wi}",
                           "--master_addr=127.0.0.1", f"--master_port={port}", str(script)] + extra,
                          env=env, timeout=180, capture_output=True)


def test_local_launch_two_ranks(tmp_path):
    r = _launch(tmp_path, [])
    assert r.returncode == 0, r.stderr.decode()[-2000:]


def test_local_launch_failure_propagates(tmp_path):
    r = _launch(tmp_path, ["--fail", "1"])
    assert r.returncode == 3


def test_env_report_runs():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bin", "ds_report")], env=dict(os.environ, PYTHONPATH=REPO),
                       capture_output=True, timeout=120)
    assert r.returncode == 0 and b"op name" in r.stdout
