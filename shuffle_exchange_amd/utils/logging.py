"""Rank-aware logging (parity: reference deepspeed/utils/logging.py:22-163)."""
import functools
import json
import logging
import os
import sys

import torch.distributed as tdist

LOG_LEVEL = os.environ.get("SXE_LOG_LEVEL", "INFO").upper()


def _make_logger():
    lg = logging.getLogger("shuffle_exchange_amd")
    if not lg.handlers:
        h = logging.StreamHandler(stream=sys.stdout)
        h.setFormatter(logging.Formatter("[%(asctime)s] [%(levelname)s] [sxe] %(message)s", "%H:%M:%S"))
        lg.addHandler(h)
    lg.setLevel(getattr(logging, LOG_LEVEL, logging.INFO))
    lg.propagate = False
    return lg


logger = _make_logger()


def _rank():
    if tdist.is_available() and tdist.is_initialized():
        return tdist.get_rank()
    return int(os.environ.get("RANK", 0))


def log_dist(message, ranks=None, level=logging.INFO):
    """Log on the given ranks only (``ranks=[-1]`` or None logs on all ranks)."""
    r = _rank()
    if ranks is None or -1 in ranks or r in ranks:
        logger.log(level, f"[Rank {r}] {message}")


@functools.lru_cache(None)
def warning_once(msg):
    logger.warning(msg)


def print_json_dist(message, ranks=None, path=None):
    r = _rank()
    if ranks is None or -1 in ranks or r in ranks:
        message["rank"] = r
        with open(path, "w") as f:
            json.dump(message, f)
            os.fsync(f)


def should_log_le(max_log_level_str):
    return logger.getEffectiveLevel() <= getattr(logging, max_log_level_str.upper())
