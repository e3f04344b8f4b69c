"""The ``autotuning`` config block (reference autotuning/config.py ``DeepSpeedAutotuningConfig`` and
autotuning/constants.py defaults) and the per-stage tuning spaces.

Tuning spaces list only knobs this framework honours (config knobs that are accepted but have no
effect -- runtime/config.py ``IGNORED_ZERO_KNOBS`` -- are never searched): ZeRO-3 prefetch /
persistence / resident-budget thresholds and the MI355X-specific deferred reduce-scatter and
retain-params schedule. ZeRO-0/1/2 have no per-stage knobs worth a run here (flat units replace
the reference's bucket sizes), so their search is over micro-batch size only.
"""
from dataclasses import dataclass, field
from typing import Optional

METRICS = ("throughput", "latency", "flops")


@dataclass
class AutotuningConfig:
    enabled: bool = False
    fast: bool = True  # True: micro-batch search only; False: also each stage's tuning space
    results_dir: str = "autotuning_results"
    exps_dir: str = "autotuning_exps"
    overwrite: bool = True
    metric: str = "throughput"
    start_profile_step: int = 3
    end_profile_step: int = 5
    tuner_type: str = "gridsearch"
    tuner_early_stopping: Optional[int] = 5
    tuner_num_trials: int = 50
    max_train_batch_size: Optional[int] = None
    min_train_micro_batch_size_per_gpu: int = 1
    max_train_micro_batch_size_per_gpu: int = 1024
    num_tuning_micro_batch_sizes: int = 3
    model_info_path: Optional[str] = None
    model_info: dict = field(default_factory=dict)
    mp_size: int = 1
    arg_mappings: dict = field(default_factory=dict)
    zero_stages: tuple = (0, 1, 2, 3)
    exp_timeout: int = 1800

    @classmethod
    def from_dict(cls, d):
        d = dict(d or {})
        known = {k: d[k] for k in cls.__dataclass_fields__ if k in d}
        if "zero_stages" in known:
            known["zero_stages"] = tuple(known["zero_stages"])
        cfg = cls(**known)
        assert cfg.metric in METRICS, f"autotuning.metric must be one of {METRICS}"
        assert cfg.end_profile_step > cfg.start_profile_step >= 0, "autotuning: end_profile_step > start_profile_step"
        return cfg


DEFAULT_TUNING_SPACE = {
    0: {},
    1: {},
    2: {},
    3: {
        "zero_optimization.stage3_param_persistence_threshold": [10_000, 100_000, 1_000_000],
        "zero_optimization.stage3_prefetch_bucket_size": [50_000_000, 500_000_000],
        "zero_optimization.stage3_defer_reduce": [False, True],
    },
}
