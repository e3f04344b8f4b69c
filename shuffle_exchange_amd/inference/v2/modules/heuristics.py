"""Implementation selection (reference inference/v2/modules/heuristics.py ``instantiate_*``): the
highest-priority registered implementation that supports the config, or a pinned one."""
from . import implementations  # noqa: F401  (registers the implementations)
from .implementations import AttentionConfig, EmbedConfig, LinearConfig, MoEConfig, NormConfig  # noqa: F401
from .registry import REGISTRIES


def _pin(pins, interface):
    return (pins or {}).get(interface)


def instantiate_linear(cfg, weight, bias=None, pins=None):
    return REGISTRIES["linear"].instantiate(cfg, weight, bias, name=_pin(pins, "linear"))


def instantiate_attention(cfg, pins=None):
    return REGISTRIES["attention"].instantiate(cfg, name=_pin(pins, "attention"))


def instantiate_moe(cfg, pins=None):
    return REGISTRIES["moe"].instantiate(cfg, name=_pin(pins, "moe"))


def instantiate_embed(cfg, weight, pins=None):
    return REGISTRIES["embed"].instantiate(cfg, weight, name=_pin(pins, "embed"))


def instantiate_norm(cfg, pins=None):
    return REGISTRIES["norm"].instantiate(cfg, name=_pin(pins, "norm"))
