"""``shuffle_exchange_amd.zero`` -- the reference's ``deepspeed.zero`` namespace."""
from .runtime.zero.partition_parameters import (Init, GatheredParameters, gather_all,  # noqa: F401
                                               register_external_parameter, unregister_external_parameter,
                                               local_shard, is_zero_param)
from .runtime.zero.stage3 import ZeroStage3Optimizer  # noqa: F401
from .runtime.zero.tiling import TiledLinear, TiledLinearReturnBias  # noqa: F401,E402
from .utils.init_on_device import OnDevice  # noqa: F401,E402
