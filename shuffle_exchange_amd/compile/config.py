"""The ``compile`` config section (reference compile/config.py ``CompileConfig``). Keys that only
make sense for the reference's Inductor pipeline (``symmetric_memory``, ``keep_*_input_tensors``,
``sync_*``, ``free_activation``, ``offload_parameters``) are accepted for config compatibility but
have no effect here -- setting one logs a warning naming it and the reason (never silent, like
runtime/config.py ``IGNORED_ZERO_KNOBS``); unknown keys warn too. The schedule passes read the rest."""
from dataclasses import dataclass, field
from typing import Optional

# accepted, no effect: key -> why (warned when set to a non-default value)
NO_EFFECT = {
    "symmetric_memory": "RCCL over xGMI needs no symmetric-memory buffers; collectives use the normal communicators",
    "sync_before_reduce": "the FX graph's reduce nodes are ordered by stream events, not host syncs",
    "sync_after_reduce": "the FX graph's reduce nodes are ordered by stream events, not host syncs",
    "sync_before_allgather": "the FX graph's gather nodes are ordered by stream events, not host syncs",
    "sync_after_allgather": "the FX graph's gather nodes are ordered by stream events, not host syncs",
    "keep_int_input_tensors": "graph inputs are never freed by the compiler",
    "keep_all_input_tensors": "graph inputs are never freed by the compiler",
    "free_activation": "activation lifetimes are autograd's; use the offload_activation pass to move them",
    "offload_parameters": "parameter offload is zero_optimization.offload_param (ZeRO-3), not a compile pass",
}


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
        cfg.ignored = cfg._warn_ignored()
        return cfg

    def _warn_ignored(self):
        from ..utils.logging import logger
        out = []
        for k, why in NO_EFFECT.items():
            if getattr(self, k) != self.__dataclass_fields__[k].default:
                out.append(k)
                logger.warning(f"config: 'compile.{k}' is accepted but has no effect: {why}")
        for k in self.extra:
            out.append(k)
            logger.warning(f"config: unknown key 'compile.{k}' ignored")
        return out
