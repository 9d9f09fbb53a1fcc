"""Logging helpers (reference parity: deepspeed/utils/logging.py:7-60)."""

import logging
import os
import sys

log_levels = {
    "debug": logging.DEBUG,
    "info": logging.INFO,
    "warning": logging.WARNING,
    "error": logging.ERROR,
    "critical": logging.CRITICAL,
}


class LoggerFactory:
    @staticmethod
    def create_logger(name=None, level=logging.INFO):
        if name is None:
            raise ValueError("name for logger cannot be None")
        formatter = logging.Formatter("[%(asctime)s] [%(levelname)s] [%(filename)s:%(lineno)d:%(funcName)s] %(message)s")
        logger_ = logging.getLogger(name)
        logger_.setLevel(level)
        logger_.propagate = False
        if not logger_.handlers:
            ch = logging.StreamHandler(stream=sys.stdout)
            ch.setLevel(level)
            ch.setFormatter(formatter)
            logger_.addHandler(ch)
        return logger_


logger = LoggerFactory.create_logger(name="DeepSpeed",
                                     level=log_levels.get(os.environ.get("DSA_LOG_LEVEL", "info"), logging.INFO))


def _rank():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    return int(os.environ.get("RANK", "0"))


def log_dist(message, ranks=None, level=logging.INFO):
    """Log `message` on the listed ranks only (-1 = all ranks)."""
    my_rank = _rank()
    if ranks is None:
        ranks = []
    if -1 in ranks or my_rank in set(ranks):
        logger.log(level, "[Rank {}] {}".format(my_rank, message))


def print_rank_0(message):
    if _rank() == 0:
        print(message, flush=True)
