"""DeepCompile counterpart (reference deepspeed/compile/): a profile-guided compiler for the ZeRO-3
step schedule. See backend.py."""
from .backend import compile_zero3, install_profiler  # noqa: F401
from .config import CompileConfig  # noqa: F401
from .graph import ScheduleGraph  # noqa: F401
from .passes import PASSES, offload_activation, offload_adam_states, prefetch, selective_gather, zero3_schedule  # noqa: F401,E501
from .profiler import ScheduleTracer  # noqa: F401
