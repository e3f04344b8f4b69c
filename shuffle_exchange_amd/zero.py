"""``shuffle_exchange_amd.zero`` -- the reference's ``deepspeed.zero`` namespace."""
from .runtime.zero.partition_parameters import Init, GatheredParameters, gather_all  # noqa: F401
from .runtime.zero.stage3 import ZeroStage3Optimizer  # noqa: F401
