from .layer import MoE  # noqa: F401
from .sharded_moe import MOELayer, TopKGate, top1gating, top2gating, topkgating  # noqa: F401
from .experts import Experts, GroupedSwiGLUExperts  # noqa: F401
from .utils import is_moe_param, split_params_into_different_moe_groups_for_optimizer  # noqa: F401
