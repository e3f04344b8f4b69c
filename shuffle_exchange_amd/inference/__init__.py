"""Inference: ``init_inference`` engine (v1 API) and the ragged FastGen-style engine (v2)."""
from .engine import InferenceConfig, InferenceEngine  # noqa: F401
