"""Inference-v2 module registry and heuristics (reference inference/v2/modules/: module_registry.py,
interfaces/*, implementations/*, heuristics.py)."""
from .heuristics import (instantiate_attention, instantiate_embed, instantiate_linear, instantiate_moe,  # noqa: F401
                         instantiate_norm)
from .registry import REGISTRIES, ModuleRegistry, register  # noqa: F401
