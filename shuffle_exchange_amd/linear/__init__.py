"""LoRA / quantized frozen-base linears (reference linear/)."""
from .optimized_linear import (LoRAConfig, LoRAOptimizedLinear, OptimizedLinear, QuantizationConfig,  # noqa: F401
                               QuantizedParameter)
