"""Packaging (reference setup.py:73-134 / install.sh): an offline, no-build-isolation pip
install ships both package names, the console scripts and the native op sources; with
DS_BUILD_OPS=0 nothing is compiled ahead of time (ops build on first use)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pip_install_offline_jit(tmp_path):
    target = tmp_path / "site"
    env = dict(os.environ, DS_BUILD_OPS="0")
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-build-isolation", "--no-index",
                        "--target", str(target), ROOT], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for script in ("deepspeed", "ds", "ds_report", "ds_elastic", "ds_ssh"):
        assert (target / "bin" / script).exists(), script
    ops = target / "deeperspeed_amd" / "ops"
    assert (ops / "csrc" / "kernels" / "flash_attn.hip").exists()
    assert (ops / "csrc" / "cpu" / "aio.cpp").exists()
    assert (target / "deepspeed" / "__init__.py").exists()
    # the installed copy imports from outside the checkout and reports its own location
    r = subprocess.run([sys.executable, "-c", "import deeperspeed_amd, deepspeed; print(deeperspeed_amd.__file__);"
                        "print(deepspeed.__version__)"], cwd=str(tmp_path),
                       env=dict(os.environ, PYTHONPATH=str(target)), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert str(target) in r.stdout and "mi355x" in r.stdout


def test_build_switches():
    sys.path.insert(0, ROOT)
    import importlib.util
    spec = importlib.util.spec_from_file_location("dsa_setup_probe", os.path.join(ROOT, "setup.py"))
    src = open(os.path.join(ROOT, "setup.py")).read().split("\nsetup(")[0]  # helpers only, no setup() call
    ns = {"__file__": os.path.join(ROOT, "setup.py")}
    exec(compile(src, "setup.py", "exec"), ns)
    old = dict(os.environ)
    try:
        for k in list(os.environ):
            if k.startswith("DS_BUILD_"):
                del os.environ[k]
        assert ns["selected_extensions"]() == ["_hip_ops", "_cpu_ops"]
        os.environ["DS_BUILD_OPS"] = "0"
        assert ns["selected_extensions"]() == []
        os.environ["DS_BUILD_CPU_ADAM"] = "1"
        assert ns["selected_extensions"]() == ["_cpu_ops"]
        os.environ["DS_BUILD_SPARSE_ATTN"] = "1"
        assert ns["selected_extensions"]() == ["_hip_ops", "_cpu_ops"]
    finally:
        os.environ.clear()
        os.environ.update(old)
    assert spec is not None
