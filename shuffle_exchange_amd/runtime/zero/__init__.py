from .partition_parameters import Init, GatheredParameters, gather_all  # noqa: F401
from .stage12 import ZeroStage12Optimizer  # noqa: F401
from .stage3 import ZeroStage3Optimizer  # noqa: F401
from .shuffle_exchange import ShuffleExchange, SliceTopology  # noqa: F401
