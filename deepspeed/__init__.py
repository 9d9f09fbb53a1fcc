"""`import deepspeed` compatibility name for deeperspeed_amd.

Every `deepspeed.<path>` import resolves to the corresponding `deeperspeed_amd` module (the
same module object, not a copy), so scripts written against DeepSpeed / DeeperSpeed
(`deepspeed.initialize`, `deepspeed.ops.adam.FusedAdam`, `deepspeed.runtime.zero.stage2`,
`deepspeed.pipe`, `deepspeed.checkpointing`, ...) run unchanged on the MI355X framework.
Reference module paths that are organised differently here are listed in _RENAMES.
"""

import importlib
import importlib.abc
import importlib.util
import sys

_TARGET = "deeperspeed_amd"
_RENAMES = {
    "deepspeed.runtime.pipe.topology": "deeperspeed_amd.runtime.pipe.topology",
    "deepspeed.ops.op_builder": "deeperspeed_amd.ops.op_builder",
    "deepspeed.op_builder": "deeperspeed_amd.ops.op_builder",
    "deepspeed.git_version_info": "deeperspeed_amd.git_version_info",
}


def _map(name):
    if name in _RENAMES:
        return _RENAMES[name]
    return _TARGET + name[len("deepspeed"):]


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith("deepspeed.") or fullname in sys.modules:
            return None
        tgt = _map(fullname)
        if importlib.util.find_spec(tgt) is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(tgt))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

_impl = importlib.import_module(_TARGET)
from deeperspeed_amd import *  # noqa: F401,F403,E402
from deeperspeed_amd import (DeepSpeedConfig, DeepSpeedEngine, __version__, add_config_arguments,  # noqa: E402
                             checkpointing, init_distributed, initialize, log_dist, logger)


# Legacy `deepspeed.pt.*` module paths (REF deepspeed/__init__.py:39-49): the same module objects
# under their pre-0.3 names.
import types as _types  # noqa: E402

_LEGACY_PT = {"deepspeed_utils": "deeperspeed_amd.runtime.utils",
              "deepspeed_config": "deeperspeed_amd.runtime.config",
              "loss_scaler": "deeperspeed_amd.runtime.fp16.loss_scaler"}
pt = _types.ModuleType("deepspeed.pt", "legacy deepspeed.pt module paths")
sys.modules["deepspeed.pt"] = pt
for _name, _target in _LEGACY_PT.items():
    _mod = importlib.import_module(_target)
    setattr(pt, _name, _mod)
    sys.modules["deepspeed.pt." + _name] = _mod


def __getattr__(name):
    return getattr(_impl, name)
