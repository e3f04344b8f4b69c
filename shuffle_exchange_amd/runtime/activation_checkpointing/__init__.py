"""Activation checkpointing (parity: reference runtime/activation_checkpointing/)."""
from . import checkpointing  # noqa: F401
from .checkpointing import (checkpoint, configure, get_cuda_rng_tracker, is_configured,  # noqa: F401
                            model_parallel_cuda_manual_seed, non_reentrant_checkpoint, reset)
