"""Package version.  The API level mirrors DeepSpeed 0.3.15 (DeeperSpeed fork), which is
what `target_deepspeed_version` checks (elasticity) and checkpoint metadata compare against."""

__version__ = "0.3.15+mi355x.1"
__version_major__ = 0
__version_minor__ = 3
__version_patch__ = 15
git_hash = "unknown"
git_branch = "main"
