"""Autotuning (reference autotuning/): tuners, the experiment scheduler and the orchestrating
Autotuner."""
from .autotuner import (Autotuner, GridSearchTuner, ModelBasedTuner, RandomTuner, model_state_bytes,  # noqa: F401
                        scheduled_runner, subprocess_runner)
from .config import DEFAULT_TUNING_SPACE, AutotuningConfig  # noqa: F401
from .scheduler import ResourceManager  # noqa: F401
