"""``FP16_UnfusedOptimizer`` (reference runtime/fp16/unfused_optimizer.py:24) -- see fused_optimizer.py."""
from .fused_optimizer import FP16_UnfusedOptimizer  # noqa: F401
