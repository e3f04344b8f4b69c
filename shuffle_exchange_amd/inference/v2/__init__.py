"""FastGen-style ragged inference (reference inference/v2/)."""
from .engine_v2 import (InferenceEngineV2, MemoryConfig, RaggedInferenceEngineConfig,  # noqa: F401
                        SchedulingError, SchedulingResult, StateManagerConfig, build_engine)
