"""Packaging for the MI355X-native DeeperSpeed framework (reference: setup.py:73-134,
install.sh).

    pip install --no-deps --no-build-isolation .          # AOT-builds the native ops for gfx950
    DS_BUILD_OPS=0 pip install --no-deps --no-build-isolation .   # JIT: ops build on first use

Native extensions: `_hip_ops` (every HIP/CDNA4 kernel: fused Adam/LAMB, transformer layer,
flash / block-sparse attention, 1-bit compression, layout transforms) and `_cpu_ops`
(AVX-512 CPU Adam, io_uring async I/O, flatten/unflatten, sparse-attention LUT utils).
The reference's per-op switches map onto them: DS_BUILD_{FUSED_ADAM,FUSED_LAMB,TRANSFORMER,
STOCHASTIC_TRANSFORMER,SPARSE_ATTN} select `_hip_ops`, DS_BUILD_{CPU_ADAM,AIO,UTILS} select
`_cpu_ops`; DS_BUILD_OPS sets the default for all of them.  Extensions not built ahead of
time are compiled in place on first import (ops/builder.py, content-hashed)."""

import os

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))

HIP_OPS = ("FUSED_ADAM", "FUSED_LAMB", "TRANSFORMER", "STOCHASTIC_TRANSFORMER", "SPARSE_ATTN")
CPU_OPS = ("CPU_ADAM", "AIO", "UTILS")


def _flag(name, default):
    v = os.environ.get(name)
    return default if v is None else v not in ("0", "false", "False", "")


def selected_extensions():
    default = _flag("DS_BUILD_OPS", True)
    out = []
    if any(_flag(f"DS_BUILD_{op}", default) for op in HIP_OPS):
        out.append("_hip_ops")
    if any(_flag(f"DS_BUILD_{op}", default) for op in CPU_OPS):
        out.append("_cpu_ops")
    return out


def _version():
    ns = {}
    with open(os.path.join(HERE, "deeperspeed_amd", "version.py")) as f:
        exec(f.read(), ns)
    return ns["__version__"]


class BuildPyWithOps(build_py):
    """Compile the selected native extensions in the source tree (gfx950), then copy the
    package -- the .so files travel as package data."""

    def run(self):
        import importlib.util
        spec = importlib.util.spec_from_file_location("_dsa_builder", os.path.join(HERE, "deeperspeed_amd", "ops",
                                                                                 "builder.py"))
        builder = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(builder)
        for name in selected_extensions():
            print(f"[deeperspeed_amd] AOT build of {name} for {builder.ARCH}")
            print("[deeperspeed_amd] built", builder.build(name))
        super().run()


setup(
    name="deeperspeed_amd",
    version=_version(),
    description="MI355X-native DeepSpeed/DeeperSpeed-compatible training engine (HIP/CDNA4 kernels, RCCL)",
    packages=find_packages(include=["deeperspeed_amd", "deeperspeed_amd.*", "deepspeed", "deepspeed.*"]),
    package_data={"deeperspeed_amd.ops": ["*.so", "*.so.hash", "csrc/*.cpp", "csrc/include/*.h", "csrc/kernels/*.hip",
                                          "csrc/cpu/*.cpp", "csrc/cpu/*.h"]},
    include_package_data=False,
    python_requires=">=3.8",
    install_requires=[],  # torch (ROCm build), numpy: provided by the environment
    entry_points={"console_scripts": [
        "deepspeed=deeperspeed_amd.launcher.runner:main",
        "deepspeed.pt=deeperspeed_amd.launcher.runner:main",
        "ds=deeperspeed_amd.launcher.runner:main",
        "ds_report=deeperspeed_amd.env_report:main",
        "ds_elastic=deeperspeed_amd.elasticity.cli:main",
    ]},
    scripts=["bin/ds_ssh"],
    cmdclass={"build_py": BuildPyWithOps},
    zip_safe=False,
)
