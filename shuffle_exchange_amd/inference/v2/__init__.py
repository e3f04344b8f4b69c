"""FastGen-style ragged inference (reference inference/v2/)."""
from .engine_v2 import (InferenceEngineV2, MemoryConfig, RaggedInferenceEngineConfig,  # noqa: F401
                        SchedulingError, SchedulingResult, StateManagerConfig, build_engine)
from .engine_factory import build_engine_from_ds_checkpoint, build_hf_engine  # noqa: F401,E402
