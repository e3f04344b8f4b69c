"""``torch_autocast`` training mode: fp32 parameters and optimizer, matmul-class modules computed
under ``torch.autocast`` in bf16 / fp16, and their gradients communicated in that lower precision.

Parity: reference runtime/torch_autocast.py:23-98 (``init_autocast_params``, the lower-precision-safe
module list, nested-autocast validation), runtime/engine.py:341-342 / 2116-2120 (forward under
``torch.autocast``) and the per-dtype gradient buckets of stage_1_and_2.py:559-563 / stage3.py:396.

MI355X design: the ZeRO optimizers here reduce whole flat units (runtime/zero/flat.py), so the
communication dtype is a property of a UNIT, not of a parameter. Stages 0-2 split every parameter
group into runs of equal communication dtype before cutting units, so the weights of the
lower-precision-safe modules (Linear / Conv) land in units that reduce-scatter / all-reduce in bf16
(half the xGMI bytes of fp32) and norms / biases of other modules stay in fp32 units. ZeRO-3 units
follow modules; a unit communicates in the autocast dtype only when every parameter in it is marked.
"""
import importlib

import torch

from ..utils.logging import logger

LOWER_PRECISION_SAFE_MODULES = [torch.nn.Linear, torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d]

_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp16": torch.float16, "float16": torch.float16,
           "half": torch.float16, "torch.bfloat16": torch.bfloat16, "torch.float16": torch.float16}

_INITIALIZED = False
_WARNED_NESTED = False


def parse_dtype(name):
    if name is None:
        return torch.bfloat16
    if isinstance(name, torch.dtype):
        return name
    key = str(name).lower()
    if key not in _DTYPES:
        raise ValueError(f"torch_autocast.dtype must be bf16 or fp16, got {name!r}")
    return _DTYPES[key]


def default_lower_precision_modules():
    return [f"{c.__module__}.{c.__name__}" for c in LOWER_PRECISION_SAFE_MODULES]


def _resolve_classes(names):
    if names is None:
        return list(LOWER_PRECISION_SAFE_MODULES)
    out = []
    for n in names:
        try:
            pkg, cls = n.rsplit(".", 1)
            out.append(getattr(importlib.import_module(pkg), cls))
        except Exception as e:
            raise ValueError(f"torch_autocast: cannot import lower-precision-safe module {n}: {e}") from e
    return out


def _is_safe(module, classes):
    # this package's own projection modules (ops/linear.Linear, the tensor-parallel layers) carry
    # ``_sxe_lower_precision_safe``; other classes match exactly, as in the reference
    if getattr(type(module), "_sxe_lower_precision_safe", False):
        return True
    return type(module) in classes


def validate(engine):
    assert not engine.fp16_enabled(), "torch_autocast cannot be combined with fp16.enabled"
    assert not engine.bfloat16_enabled(), "torch_autocast cannot be combined with bf16.enabled"
    zc = engine._config.zero_config
    assert not zc.zero_quantized_weights, "torch_autocast cannot be combined with zero_quantized_weights"
    bad = [n for n, p in engine.module.named_parameters() if p.dtype != torch.float32]
    assert not bad, f"torch_autocast needs float32 parameters (not: {bad[:4]})"
    cdt = engine.communication_data_type
    assert cdt in (None, torch.float32), "torch_autocast: communication_data_type must be fp32 (or unset)"


def init_autocast_params(engine, dtype, safe_module_names=None):
    """Mark the parameters of lower-precision-safe modules with ``autocast_dtype`` (their gradients
    are communicated in that dtype). Returns the number of marked parameters."""
    global _INITIALIZED
    validate(engine)
    classes = _resolve_classes(safe_module_names)
    n = 0
    for m in engine.module.modules():
        if _is_safe(m, classes):
            for p in m.parameters(recurse=False):
                p.autocast_dtype = dtype
                n += 1
    _INITIALIZED = True
    logger.info(f"torch_autocast: {dtype}, {n} parameters of lower-precision-safe modules communicate in {dtype}")
    return n


def is_autocast_initialized():
    return _INITIALIZED


def get_autocast_dtype(param):
    return getattr(param, "autocast_dtype", param.dtype)


def has_autocast_dtype(param):
    return hasattr(param, "autocast_dtype")


def comm_dtype_of(param, default=None):
    """Gradient communication dtype of one parameter: its autocast dtype when marked."""
    return getattr(param, "autocast_dtype", default)


def unit_comm_dtype(params, default=None):
    """A flat unit's communication dtype: the autocast dtype when EVERY parameter carries the same
    one, else ``default`` (fp32 reduction keeps the unmarked parameters exact)."""
    dts = {getattr(p, "autocast_dtype", None) for p in params}
    if len(dts) == 1:
        d = dts.pop()
        if d is not None:
            return d
    return default


def split_by_comm_dtype(params):
    """Stable partition of a parameter list into runs of equal communication dtype (autocast-marked
    first, then the rest), so flat units never mix the two."""
    marked = [p for p in params if has_autocast_dtype(p)]
    rest = [p for p in params if not has_autocast_dtype(p)]
    return [grp for grp in (marked, rest) if grp]


def validate_nested_autocast(engine):
    """Reference torch_autocast.py:86-98: an outer torch.autocast is redundant when the config enables
    it (warn once) and an error when it does not (the gradients would travel in the wrong dtype)."""
    global _WARNED_NESTED
    if not torch.is_autocast_enabled(engine.device.type):
        return
    if engine.torch_autocast_enabled():
        if not _WARNED_NESTED:
            logger.warning("torch.autocast is already enabled through the config; the outer context is redundant")
            _WARNED_NESTED = True
    else:
        raise AssertionError("torch.autocast is enabled outside the engine but not in the config: enable "
                             "'torch_autocast' in the config so gradients are communicated in the right dtype")
