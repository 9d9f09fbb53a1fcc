"""Build/version information at the reference's import path (deepspeed/git_version_info.py)."""

import os
import subprocess

from .version import __version__ as version


def _git(*args):
    try:
        return subprocess.check_output(["git", *args], cwd=os.path.dirname(os.path.abspath(__file__)),
                                       stderr=subprocess.DEVNULL).decode().strip()
    except Exception:
        return "unknown"


git_hash = _git("rev-parse", "--short", "HEAD")
git_branch = _git("rev-parse", "--abbrev-ref", "HEAD")


def _ops():
    from .ops import op_builder
    ref = {"FusedAdamBuilder": "fused_adam", "FusedLambBuilder": "fused_lamb", "TransformerBuilder": "transformer",
           "StochasticTransformerBuilder": "stochastic_transformer", "SparseAttnBuilder": "sparse_attn",
           "CPUAdamBuilder": "cpu_adam", "AsyncIOBuilder": "async_io", "UtilsBuilder": "utils"}
    return [ref.get(k, k) for k in getattr(op_builder, "ALL_OPS", {})]


try:
    _names = _ops()
except Exception:
    _names = []
# ops are compiled in-tree on first use (ops/builder.py), so every op is "installed" once built
installed_ops = {n: True for n in _names}
compatible_ops = {n: True for n in _names}
