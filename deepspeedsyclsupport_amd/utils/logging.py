"""Rank-aware logging (`deepspeed/utils/logging.py` parity: `logger`, `log_dist`, `print_json_dist`)."""
import json
import logging
import os
import sys

import torch.distributed as dist

_FMT = "[%(asctime)s] [%(levelname)s] [%(filename)s:%(lineno)d:%(funcName)s] %(message)s"


def _create_logger(name="DeepSpeedAMD", level=logging.INFO):
    lg = logging.getLogger(name)
    lg.setLevel(level)
    lg.propagate = False
    if not lg.handlers:
        h = logging.StreamHandler(stream=sys.stdout)
        h.setFormatter(logging.Formatter(_FMT))
        lg.addHandler(h)
    return lg


class LoggerFactory:
    """Named loggers with the package's format (reference `utils/logging.py:LoggerFactory`)."""

    @staticmethod
    def create_logger(name=None, level=logging.INFO):
        if name is None:
            raise ValueError("name for logger cannot be None")
        return _create_logger(name, level)


logger = _create_logger(level=getattr(logging, os.environ.get("DS_LOG_LEVEL", "INFO").upper(), logging.INFO))


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def log_dist(message, ranks=None, level=logging.INFO):
    """Log on the listed ranks only (None or [-1] means every rank)."""
    my = _rank()
    if ranks is None or -1 in ranks or my in ranks:
        logger.log(level, f"[Rank {my}] {message}")


def print_json_dist(message, ranks=None, path=None):
    my = _rank()
    if ranks is None or -1 in ranks or my in ranks:
        message["rank"] = my
        with open(path, "w") as f:
            json.dump(message, f)
            os.fsync(f)


def should_log_le(max_log_level_str):
    return logger.getEffectiveLevel() <= getattr(logging, max_log_level_str.upper())


import functools


@functools.lru_cache(None)
def warning_once(*args, **kwargs):
    """`logger.warning` that fires once per distinct message."""
    logger.warning(*args, **kwargs)


logger.warning_once = warning_once


def print_configuration(args, name):
    logger.info("{}:".format(name))
    for arg in sorted(vars(args)):
        logger.info("  {} {} {}".format(arg, "." * (29 - len(arg)), getattr(args, arg)))


def get_current_level():
    return logger.getEffectiveLevel()

