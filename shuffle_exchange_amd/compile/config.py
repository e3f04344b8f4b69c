"""The ``compile`` config section (reference compile/config.py ``CompileConfig``). Keys that only
make sense for an FX/Inductor pipeline (``symmetric_memory``, ``keep_*_input_tensors``,
``sync_*``) are accepted and have no effect; the schedule passes read the rest."""
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class CompileConfig:
    deepcompile: bool = False
    free_activation: bool = False
    offload_activation: bool = False
    offload_opt_states: bool = False
    double_buffer: bool = True
    symmetric_memory: bool = False
    debug_log: bool = False
    offload_parameters: bool = False
    sync_before_reduce: bool = False
    sync_after_reduce: bool = False
    sync_before_allgather: bool = False
    sync_after_allgather: bool = False
    keep_int_input_tensors: bool = True
    keep_all_input_tensors: bool = False
    # schedule compiler (this framework)
    passes: tuple = ("selective_gather", "prefetch", "offload_adam_states", "offload_activation")
    memory_budget: Optional[float] = None   # bytes (> 1) or a fraction of device memory (<= 1); default 0.9
    profile_steps: int = 1                  # optimizer steps traced before the passes run
    prefetch_slack: float = 1.25            # gather-time safety factor when placing prefetches
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_dict(cls, d):
        d = dict(d or {})
        known = {k: d.pop(k) for k in list(d) if k in cls.__dataclass_fields__}
        if "passes" in known:
            known["passes"] = tuple(known["passes"])
        cfg = cls(**known)
        cfg.extra = d
        return cfg
