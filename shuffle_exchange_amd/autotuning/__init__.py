"""Autotuning (reference autotuning/)."""
from .autotuner import (Autotuner, GridSearchTuner, ModelBasedTuner, RandomTuner, model_state_bytes,  # noqa: F401
                        subprocess_runner)
