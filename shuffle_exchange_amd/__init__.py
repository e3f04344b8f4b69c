"""shuffle_exchange_amd -- an MI355X-native (ROCm / gfx950) distributed training & inference framework
with the capabilities of vituslcx/Shuffle-exchange (a DeepSpeed snapshot + hierarchical
"Shuffle-exchange" ZeRO).

Public API mirrors the reference (deepspeed/__init__.py:69 ``initialize``, :299 ``init_inference``,
:276 ``add_config_arguments``) including the fork's ``shuffle_step / rings / method / slice_count``
keyword arguments (deepspeed/__init__.py:82-85).
"""
import argparse

from . import comm  # noqa: F401
from . import zero  # noqa: F401
from .accelerator import get_accelerator  # noqa: F401
from .comm import init_distributed  # noqa: F401
from .runtime.config import SXEConfig, DeepSpeedConfig  # noqa: F401
from .runtime.engine import SXEEngine  # noqa: F401
from .runtime import lr_schedules  # noqa: F401
from .runtime.activation_checkpointing import checkpointing  # noqa: F401
from .utils.logging import logger, log_dist  # noqa: F401
from .utils.init_on_device import OnDevice  # noqa: F401
from .runtime.utils import see_memory_usage  # noqa: F401
from .ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer  # noqa: F401

__version__ = "0.1.0"
__git_branch__ = "main"

DeepSpeedEngine = SXEEngine


def initialize(args=None, model=None, optimizer=None, model_parameters=None, training_data=None, lr_scheduler=None,
               distributed_port=29500, mpu=None, dist_init_required=None, collate_fn=None, config=None,
               mesh_param=None, config_params=None, shuffle_step=None, rings=None, method=None, slice_count=None):
    """Build the training engine. Returns ``(engine, optimizer, training_dataloader, lr_scheduler)``.

    ``shuffle_step / rings / method / slice_count`` enable Shuffle-exchange hierarchical ZeRO
    (the reference applies them to ZeRO-1/2 only; here they also apply to ZeRO-3). They can also be
    given as a ``"shuffle_exchange"`` block in the config.
    """
    assert model is not None, "initialize() requires a model"
    if config is None:
        config = config_params
    if config is None and args is not None:
        config = getattr(args, "deepspeed_config", None) or getattr(args, "sxe_config", None)
    init_distributed(distributed_port=distributed_port, dist_init_required=dist_init_required)
    config, mesh_device = _mesh_from_args(config, mesh_param)
    pp = getattr(model, "is_pipeline_module", False)
    if pp:
        from .runtime.pipe.engine import PipelineEngine
        engine = PipelineEngine(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                                training_data=training_data, lr_scheduler=lr_scheduler, mpu=model.mpu(),
                                dist_init_required=dist_init_required, collate_fn=collate_fn, config=config)
    else:
        cls = SXEEngine
        try:
            from .runtime.config import _load_raw
            if _load_raw(config).get("hybrid_engine", {}).get("enabled", False):
                from .runtime.hybrid_engine import SXEHybridEngine
                cls = SXEHybridEngine
        except Exception:
            pass
        engine = cls(args=args, model=model, optimizer=optimizer, model_parameters=model_parameters,
                           training_data=training_data, lr_scheduler=lr_scheduler, mpu=mpu,
                           dist_init_required=dist_init_required, collate_fn=collate_fn, config=config,
                           rings=rings, shuffle_step=shuffle_step, method=method, slice_count=slice_count,
                           mesh_device=mesh_device)
    return engine, engine.optimizer, engine.training_dataloader, engine.lr_scheduler


def _mesh_from_args(config, mesh_param):
    """``mesh_param=(dp, sp)`` -- or both ``data_parallel_size`` and ``sequence_parallel_size`` in the
    config -- builds a 2-D ("data_parallel", "sequence_parallel") DeviceMesh over the world and sets
    the engine's sequence-parallel size from it (reference deepspeed/__init__.py:157-166)."""
    from .runtime.config import _load_raw
    raw = _load_raw(config) if config is not None else {}
    if mesh_param is not None:
        dp, sp = (int(x) for x in mesh_param)
    elif "data_parallel_size" in raw and "sequence_parallel_size" in raw:
        dp, sp = int(raw["data_parallel_size"]), int(raw["sequence_parallel_size"])
    else:
        return config, None
    world = comm.get_world_size()
    if dp * sp != world:
        raise ValueError(f"mesh (dp={dp}, sp={sp}) does not cover the world of {world} ranks")
    if raw.get("sequence_parallel_size", sp) != sp:
        raise ValueError(f"mesh_param sp={sp} contradicts sequence_parallel_size={raw['sequence_parallel_size']}")
    raw["sequence_parallel_size"] = sp
    raw["data_parallel_size"] = dp
    raw.pop("mesh_param", None)
    logger.info(f"mesh: data_parallel={dp} x sequence_parallel={sp}")
    return raw, comm.initialize_mesh_device((dp, sp), ("data_parallel", "sequence_parallel"))


def add_config_arguments(parser):
    group = parser.add_argument_group("shuffle_exchange_amd", "configuration")
    group.add_argument("--deepspeed", default=False, action="store_true", help="enable the engine")
    group.add_argument("--deepspeed_config", default=None, type=str, help="JSON config path")
    group.add_argument("--sxe_config", default=None, type=str, help="alias of --deepspeed_config")
    return parser


def add_core_arguments(parser):
    return add_config_arguments(parser)


def init_inference(model, config=None, **kwargs):
    from .inference.engine import InferenceEngine, InferenceConfig
    cfg = InferenceConfig(**{**(config or {}), **kwargs}) if not isinstance(config, InferenceConfig) else config
    return InferenceEngine(model, cfg)


def _parse_args(argv=None):
    p = argparse.ArgumentParser()
    add_config_arguments(p)
    return p.parse_args(argv)
