"""deeperspeed_amd: an MI355X-native ZeRO + 3D-parallel training engine with the capabilities
and API of DeeperSpeed (DeepSpeed v0.3.15 lineage).

Public API (reference parity: deepspeed/__init__.py:52-212):
    initialize(args, model, optimizer, model_parameters, training_data, lr_scheduler, mpu,
               dist_init_required, collate_fn, config_params)
        -> (engine, optimizer, training_dataloader, lr_scheduler)
    add_config_arguments(parser), init_distributed(...)
"""

import argparse
import sys
import types

from .version import __version__, git_branch as __git_branch__, git_hash as __git_hash__
from .utils.logging import log_dist, logger
from .utils.distributed import init_distributed
from .runtime.config import DeepSpeedConfig
from .runtime.engine import DeepSpeedEngine
from .runtime.activation_checkpointing import checkpointing
from .runtime import lr_schedules
from .runtime.dataloader import RepeatingLoader


def _parse_version(version_str):
    import re
    m = re.search(r"^(\d+)\.(\d+)\.(\d+)", version_str)
    return int(m.group(1)), int(m.group(2)), int(m.group(3))


__version_major__, __version_minor__, __version_patch__ = _parse_version(__version__)


def _pipeline_classes():
    from .runtime.pipe.engine import PipelineEngine
    from .runtime.pipe.module import PipelineModule
    return PipelineEngine, PipelineModule


def initialize(args=None, model=None, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
               mpu=None, dist_init_required=None, collate_fn=None, config_params=None):
    """Build a DeepSpeedEngine (or PipelineEngine for a PipelineModule) around `model`.

    Returns (engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler).
    """
    log_dist("DeepSpeed info: version={}, git-hash={}, git-branch={}".format(__version__, __git_hash__,
                                                                              __git_branch__), ranks=[0])
    assert model is not None, "deepspeed.initialize requires a model"
    PipelineEngine, PipelineModule = _pipeline_classes()
    if not isinstance(model, PipelineModule):
        engine = DeepSpeedEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                 training_data=training_data, lr_scheduler=lr_scheduler, mpu=mpu,
                                 dist_init_required=dist_init_required, collate_fn=collate_fn,
                                 config_params=config_params)
    else:
        assert mpu is None, "mpu must be None with pipeline parallelism"
        engine = PipelineEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                training_data=training_data, lr_scheduler=lr_scheduler, mpu=model.mpu(),
                                dist_init_required=dist_init_required, collate_fn=collate_fn,
                                config_params=config_params)
    return engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler


def _add_core_arguments(parser):
    group = parser.add_argument_group("DeepSpeed", "DeepSpeed configurations")
    group.add_argument("--deepspeed", default=False, action="store_true",
                       help="Enable DeepSpeed (helper flag for user code, no impact on DeepSpeed backend)")
    group.add_argument("--deepspeed_config", default=None, type=str, help="DeepSpeed json configuration file.")
    group.add_argument("--deepscale", default=False, action="store_true",
                       help="Deprecated enable DeepSpeed (helper flag for user code, no impact on DeepSpeed backend)")
    group.add_argument("--deepscale_config", default=None, type=str,
                       help="Deprecated DeepSpeed json configuration file.")
    group.add_argument("--deepspeed_mpi", default=False, action="store_true",
                       help="Run via MPI, this will attempt to discover the necessary variables to initialize "
                            "torch distributed from the MPI environment")
    return parser


def add_config_arguments(parser):
    """Update the argument parser to enable parsing of DeepSpeed command line arguments."""
    return _add_core_arguments(parser)


def __getattr__(name):
    # lazy attributes that import heavier subsystems on first use
    if name in ("PipelineEngine", "PipelineModule"):
        pe, pm = _pipeline_classes()
        return pe if name == "PipelineEngine" else pm
    if name in ("pipe", "zero", "ops", "profiling", "elasticity", "module_inject", "launcher", "models", "parallel"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    if name in ("DeepSpeedTransformerLayer", "DeepSpeedTransformerConfig"):
        from .ops import transformer
        return getattr(transformer, name)
    raise AttributeError(name)
