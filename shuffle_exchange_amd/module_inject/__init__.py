"""Tensor-parallel layer injection (parity: reference module_inject/)."""
from .auto_tp import AutoTP, gather_tp_state_dict, tp_model_init  # noqa: F401
from .layers import (GatherReplacedLayerParams, LinearAllreduce, LinearLayer, LmHeadLinearAllreduce,  # noqa: F401
                     TensorParallelLinearBase)
from .diffusers import FusedDiffusersAttention, generic_injection  # noqa: F401,E402
