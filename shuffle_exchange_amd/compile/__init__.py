"""DeepCompile counterpart (reference deepspeed/compile/): an FX graph compiler for ZeRO 0/1/2
(fx_backend.py, fx_graph.py: in-graph gradient reduction) and a profile-guided compiler for the
ZeRO-3 step schedule (backend.py, passes.py)."""
from .backend import compile_zero3, install_profiler  # noqa: F401
from .config import CompileConfig  # noqa: F401
from .graph import ScheduleGraph  # noqa: F401
from .passes import PASSES, offload_activation, offload_adam_states, prefetch, selective_gather, zero3_schedule  # noqa: F401,E501
from .profiler import ScheduleTracer  # noqa: F401
from .fx_backend import FXCompiler, compile_fx  # noqa: F401
