"""``BF16_Optimizer`` (reference runtime/bf16_optimizer.py:35) -- see runtime/fp16/fused_optimizer.py."""
from .fp16.fused_optimizer import BF16_Optimizer  # noqa: F401
