from .logging import log_dist, logger
from .distributed import init_distributed


def __getattr__(name):
    if name == "RepeatingLoader":
        from ..runtime.dataloader import RepeatingLoader
        return RepeatingLoader
    raise AttributeError(name)
