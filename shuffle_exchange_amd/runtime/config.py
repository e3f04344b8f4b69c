"""Typed configuration (JSON/dict/base64 -> pydantic models).

Parity: reference runtime/config.py:648-997 (``DeepSpeedConfig``; batch-triple solve :870-936),
runtime/config_utils.py:17-80 (pydantic base with deprecated-alias handling), runtime/zero/config.py:86-344
and runtime/zero/offload_config.py:21-100. The JSON keys are the reference's, so existing configs
load unchanged. New: a ``shuffle_exchange`` block (the fork's knobs are kwargs-only in the
reference, __init__.py:82-85) -- kwargs still win when both are given.
"""
import base64
import copy
import json
import os
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, ConfigDict, Field, model_validator

from ..utils.logging import logger


class ConfigModel(BaseModel):
    """Base: deprecated aliases map to their new field. Unknown keys are collected by
    ``SXEConfig._check_unknown_keys`` after parsing: a warning naming the key (with the closest
    known field) by default, a ``ValueError`` with ``"strict_config": true`` or SXE_STRICT_CONFIG=1
    (the reference forbids extras in every block, runtime/config_utils.py:110 ``extra="forbid"``)."""
    model_config = ConfigDict(extra="allow", populate_by_name=True, validate_assignment=True,
                              arbitrary_types_allowed=True, protected_namespaces=())


# ---------------------------------------------------------------------------------------------- ZeRO
class OffloadDeviceEnum:
    none = "none"
    cpu = "cpu"
    nvme = "nvme"


class OffloadConfig(ConfigModel):
    device: str = "none"
    nvme_path: Optional[str] = None
    buffer_count: int = 5
    buffer_size: int = 100_000_000
    max_in_cpu: int = 1_000_000_000
    pin_memory: bool = False
    pipeline_read: bool = False
    pipeline_write: bool = False
    fast_init: bool = False
    ratio: float = 1.0


class ZeroConfig(ConfigModel):
    stage: int = 0
    contiguous_gradients: bool = True
    reduce_scatter: bool = True
    reduce_bucket_size: int = 500_000_000
    use_multi_rank_bucket_allreduce: bool = True
    allgather_partitions: bool = True
    allgather_bucket_size: int = 500_000_000
    overlap_comm: Optional[bool] = None
    load_from_fp32_weights: bool = True
    elastic_checkpoint: bool = False
    offload_param: Optional[OffloadConfig] = None
    offload_optimizer: Optional[OffloadConfig] = None
    sub_group_size: int = 1_000_000_000
    cpu_offload: Optional[bool] = None
    prefetch_bucket_size: int = Field(50_000_000, alias="stage3_prefetch_bucket_size")
    param_persistence_threshold: int = Field(100_000, alias="stage3_param_persistence_threshold")
    model_persistence_threshold: int = Field(2**63 - 1, alias="stage3_model_persistence_threshold")
    max_live_parameters: int = Field(1_000_000_000, alias="stage3_max_live_parameters")
    max_reuse_distance: int = Field(1_000_000_000, alias="stage3_max_reuse_distance")
    gather_16bit_weights_on_model_save: bool = Field(False, alias="stage3_gather_16bit_weights_on_model_save")
    module_granularity_threshold: int = 0
    ignore_unused_parameters: bool = True
    legacy_stage1: bool = False
    round_robin_gradients: bool = False
    zero_hpz_partition_size: int = 1
    zero_quantized_weights: bool = False
    zero_quantized_nontrainable_weights: bool = False
    zero_quantized_gradients: bool = False
    zeropp_loco_param: Optional[Dict[str, Any]] = None  # {"err_beta": 0.8, "reset_T": 1024}: LoCo error feedback
    mics_shard_size: int = -1
    mics_hierarchical_params_gather: bool = False
    memory_efficient_linear: bool = True
    pipeline_loading_checkpoint: bool = False
    override_module_apply: bool = True
    log_trace_cache_warnings: bool = False
    # MI355X-specific knobs (new): units of ZeRO-3 fetch (module class names) and prefetch depth
    fetch_units: Optional[List[str]] = None
    prefetch_depth: int = 2
    # MI355X (288 GB HBM): ZeRO-3 keeps each unit's fp32 gradient sum across the micro-steps of one
    # optimizer step and reduce-scatters once at the accumulation boundary
    defer_reduce: bool = Field(False, alias="stage3_defer_reduce")
    # ... and keeps gathered parameters resident across those micro-steps (one all-gather per step)
    retain_params: bool = Field(False, alias="stage3_retain_params_in_step")

    @model_validator(mode="after")
    def _compat(self):
        if self.cpu_offload and self.offload_optimizer is None:
            self.offload_optimizer = OffloadConfig(device="cpu", pin_memory=True)
        if self.overlap_comm is None:
            object.__setattr__(self, "overlap_comm", self.stage == 3)
        return self


class ShuffleExchangeConfig(ConfigModel):
    """The fork's hierarchical ZeRO-1/2 knobs (reference __init__.py:82-85, stage_1_and_2.py:163-241)."""
    enabled: bool = False
    method: str = "RR"           # RR | shuffle | H-RR | Gossip
    slice_count: int = 2         # ranks per ZeRO slice (the ZeRO partition group)
    rings: int = 8               # ring groups for `shuffle` (forced to 2 for H-RR)
    shuffle_step: int = 50       # reshuffle period in shuffle_exchange() calls
    seed: int = 1234             # seeds the rank-consistent permutation generator
    sync_period: int = 0         # >0: engine calls synchronization() every N steps (new)
    gossip_p: float = 1.0        # Bernoulli send probability for Gossip
    auto_shuffle: bool = False   # engine calls shuffle_exchange() after every step (new)

    @model_validator(mode="after")
    def _check(self):
        m = self.method
        if m not in ("RR", "shuffle", "H-RR", "Gossip"):
            raise ValueError(f"shuffle_exchange.method must be RR|shuffle|H-RR|Gossip, got {m}")
        if self.slice_count < 1:
            raise ValueError("shuffle_exchange.slice_count must be >= 1")
        return self


# ------------------------------------------------------------------------------------------ precision
class FP16Config(ConfigModel):
    enabled: bool = False
    auto_cast: bool = False
    loss_scale: float = 0.0
    initial_scale_power: int = 16
    loss_scale_window: int = 1000
    hysteresis: int = 2
    consecutive_hysteresis: bool = False
    min_loss_scale: float = 1.0
    fp16_master_weights_and_grads: bool = False


class BF16Config(ConfigModel):
    enabled: bool = False
    immediate_grad_update: bool = False
    check_grad_overflow: bool = False


class DataTypesConfig(ConfigModel):
    # None: the reference default (fp32 for bf16 without ZeRO, else the model dtype,
    # reference runtime/engine.py:1074-1089); "fp32" with bf16 ZeRO-1 = BF16_Optimizer semantics
    grad_accum_dtype: Optional[str] = None

    @model_validator(mode="after")
    def _check(self):
        if self.grad_accum_dtype is not None and self.grad_accum_dtype not in ("fp32", "fp16", "bf16", "float32",
                                                                                 "float16", "bfloat16"):
            raise ValueError(f"data_types.grad_accum_dtype must be fp32|fp16|bf16, got {self.grad_accum_dtype}")
        return self


class OptimizerConfig(ConfigModel):
    type: str = "AdamW"
    params: Dict[str, Any] = Field(default_factory=dict)
    legacy_fusion: bool = False


class SchedulerConfig(ConfigModel):
    type: Optional[str] = None
    params: Dict[str, Any] = Field(default_factory=dict)


# ---------------------------------------------------------------------------------------------- misc
class ActivationCheckpointingConfig(ConfigModel):
    partition_activations: bool = False
    contiguous_memory_optimization: bool = False
    cpu_checkpointing: bool = False
    number_checkpoints: Optional[int] = None
    synchronize_checkpoint_boundary: bool = False
    profile: bool = False


class CommsLoggerConfig(ConfigModel):
    enabled: bool = False
    verbose: bool = False
    prof_all: bool = True
    debug: bool = False
    prof_ops: List[str] = Field(default_factory=list)


class FlopsProfilerConfig(ConfigModel):
    enabled: bool = False
    recompute_fwd_factor: float = 0.0
    profile_step: int = 1
    module_depth: int = -1
    top_modules: int = 1
    detailed: bool = True
    output_file: Optional[str] = None


class TensorBoardConfig(ConfigModel):
    enabled: bool = False
    output_path: str = ""
    job_name: str = "SXEJobName"


class CSVConfig(ConfigModel):
    enabled: bool = False
    output_path: str = ""
    job_name: str = "SXEJobName"


class WandbConfig(ConfigModel):
    enabled: bool = False
    group: Optional[str] = None
    team: Optional[str] = None
    project: str = "shuffle_exchange_amd"


class CometConfig(ConfigModel):
    enabled: bool = False
    project: Optional[str] = None
    experiment_name: Optional[str] = None


class CheckpointConfig(ConfigModel):
    tag_validation: str = "WARN"
    load_universal: bool = False
    use_node_local_storage: bool = False
    parallel_write: Dict[str, Any] = Field(default_factory=dict)
    writer: Optional[Dict[str, Any]] = None
    async_save: bool = False  # decoupled (background) checkpoint engine


class AIOConfig(ConfigModel):
    block_size: int = 1 << 20
    queue_depth: int = 8
    intra_op_parallelism: int = Field(4, alias="thread_count")
    single_submit: bool = False
    overlap_events: bool = True
    use_gds: bool = False


class PipelineConfig(ConfigModel):
    stages: Any = "auto"
    partition: str = "parameters"
    seed_layers: bool = False
    activation_checkpoint_interval: int = 0
    pipe_partitioned: bool = True
    grad_partitioned: bool = True


class HybridEngineConfig(ConfigModel):
    enabled: bool = False
    max_out_tokens: int = 512
    inference_tp_size: int = 1
    release_inference_cache: bool = False
    pin_parameters: bool = True
    tp_gather_partition_size: int = 8
    kv_cache_fraction: float = 0.3


class TensorParallelConfig(ConfigModel):
    autotp_size: int = 1
    tp_size: int = 1


class ElasticityConfig(ConfigModel):
    enabled: bool = False
    max_train_batch_size: int = 2000
    micro_batch_sizes: List[int] = Field(default_factory=lambda: [2, 4, 6])
    min_gpus: int = 1
    max_gpus: int = 10000
    min_time: int = 20
    version: float = 0.2
    ignore_non_elastic_batch_info: bool = False
    prefer_larger_batch: bool = True
    num_gpus_per_node: int = 8
    model_parallel_size: int = 1


class TorchAutocastConfig(ConfigModel):
    """Reference runtime/constants.py:217-226 ``torch_autocast`` block (runtime/torch_autocast.py)."""
    enabled: bool = False
    dtype: Optional[str] = None  # bf16 (default) or fp16
    lower_precision_safe_modules: Optional[List[str]] = None


class MoEConfig(ConfigModel):
    ep_size: int = 1
    drop_tokens: bool = True
    capacity_factor: float = 1.0


# ---------------------------------------------------------------------------------------------- root
class SXEConfigModel(ConfigModel):
    train_batch_size: Optional[int] = None
    train_micro_batch_size_per_gpu: Optional[int] = None
    gradient_accumulation_steps: Optional[int] = None
    steps_per_print: int = 10
    dump_state: bool = False
    gradient_clipping: float = 0.0
    prescale_gradients: bool = False
    gradient_predivide_factor: float = 1.0
    sparse_gradients: bool = False
    wall_clock_breakdown: bool = False
    memory_breakdown: bool = False
    zero_allow_untested_optimizer: bool = False
    zero_force_ds_cpu_optimizer: bool = True
    communication_data_type: Optional[str] = None
    seq_parallel_communication_data_type: str = "fp32"
    sequence_parallel_size: int = 1
    data_parallel_size: Optional[int] = None
    pipeline_parallel_size: int = 1
    seed: int = 1234
    disable_allgather: bool = False
    graph_harvesting: bool = False
    use_data_before_expert_parallel_: bool = False
    zero_optimization: ZeroConfig = Field(default_factory=ZeroConfig)
    shuffle_exchange: ShuffleExchangeConfig = Field(default_factory=ShuffleExchangeConfig)
    fp16: FP16Config = Field(default_factory=FP16Config)
    bf16: BF16Config = Field(default_factory=BF16Config)
    data_types: DataTypesConfig = Field(default_factory=DataTypesConfig)
    optimizer: Optional[OptimizerConfig] = None
    scheduler: Optional[SchedulerConfig] = None
    activation_checkpointing: ActivationCheckpointingConfig = Field(default_factory=ActivationCheckpointingConfig)
    comms_logger: CommsLoggerConfig = Field(default_factory=CommsLoggerConfig)
    flops_profiler: FlopsProfilerConfig = Field(default_factory=FlopsProfilerConfig)
    tensorboard: TensorBoardConfig = Field(default_factory=TensorBoardConfig)
    csv_monitor: CSVConfig = Field(default_factory=CSVConfig)
    wandb: WandbConfig = Field(default_factory=WandbConfig)
    comet: CometConfig = Field(default_factory=CometConfig)
    checkpoint: CheckpointConfig = Field(default_factory=CheckpointConfig)
    aio: AIOConfig = Field(default_factory=AIOConfig)
    pipeline: PipelineConfig = Field(default_factory=PipelineConfig)
    tensor_parallel: TensorParallelConfig = Field(default_factory=TensorParallelConfig)
    hybrid_engine: HybridEngineConfig = Field(default_factory=HybridEngineConfig)
    elasticity: ElasticityConfig = Field(default_factory=ElasticityConfig)
    moe: MoEConfig = Field(default_factory=MoEConfig)
    torch_autocast: TorchAutocastConfig = Field(default_factory=TorchAutocastConfig)
    amp: Dict[str, Any] = Field(default_factory=dict)
    compile: Dict[str, Any] = Field(default_factory=dict)
    strict_config: bool = False  # new: unknown keys raise instead of warning


# Root blocks consumed from the raw dict by their own subsystems (engine / data pipeline / compression
# / autotuning / sparse attention ...), plus reference root keys accepted for compatibility.
RAW_ROOT_KEYS = {
    "data_efficiency", "curriculum_learning", "progressive_layer_drop", "quantize_training", "autotuning",
    "compression_training", "sparse_attention", "eigenvalue", "weight_quantization", "dataloader_drop_last",
    "bfloat16", "nebula", "monitor_config", "data_sampling", "zero_enabled", "deepcompile",
    "timers", "use_node_local_storage", "pipeline_stage", "inference", "mesh_param",
}


def _load_raw(config):
    if config is None:
        return {}
    if isinstance(config, dict):
        return copy.deepcopy(config)
    if isinstance(config, str):
        if os.path.exists(config):
            with open(config) as f:
                return json.load(f, object_pairs_hook=_no_dup)
        try:
            return json.loads(base64.urlsafe_b64decode(config).decode(), object_pairs_hook=_no_dup)
        except Exception as e:
            raise ValueError(f"config '{config[:64]}' is neither a file nor base64 JSON") from e
    raise TypeError(f"unsupported config type {type(config)}")


def _no_dup(pairs):
    d = {}
    for k, v in pairs:
        if k in d:
            raise ValueError(f"duplicate key in config: {k}")
        d[k] = v
    return d


class SXEConfig:
    """Resolved configuration. ``world_size`` is the *data-parallel* world (world / (tp*pp*sp))."""

    def __init__(self, config, world_size=1, mpu=None, tp_size=1, pp_size=1):
        raw = _load_raw(config)
        self._param_dict = raw
        self.model = SXEConfigModel(**raw)
        m = self.model
        sp = max(1, m.sequence_parallel_size)
        tp = max(tp_size, m.tensor_parallel.autotp_size, m.tensor_parallel.tp_size)
        pp = max(pp_size, m.pipeline_parallel_size)
        if mpu is not None and hasattr(mpu, "get_data_parallel_world_size"):
            self.dp_world_size = mpu.get_data_parallel_world_size()
        else:
            assert world_size % (tp * sp * pp) == 0, "world size must be divisible by tp*sp*pp"
            self.dp_world_size = world_size // (tp * sp * pp)
        self.world_size = world_size
        self.sequence_parallel_size = sp
        self.tensor_parallel_size = tp
        self.pipeline_parallel_size = pp
        self._solve_batch()
        # flat attribute views used across the runtime
        self.zero_config = m.zero_optimization
        self.zero_optimization_stage = m.zero_optimization.stage
        self.zero_enabled = self.zero_optimization_stage > 0
        self.fp16_enabled = m.fp16.enabled
        self.bfloat16_enabled = m.bf16.enabled
        self.gradient_clipping = m.gradient_clipping
        self.steps_per_print = m.steps_per_print
        self.wall_clock_breakdown = m.wall_clock_breakdown
        self.shuffle_exchange = m.shuffle_exchange
        self.optimizer_name = m.optimizer.type.lower() if m.optimizer else None
        self.optimizer_params = dict(m.optimizer.params) if m.optimizer else {}
        self.scheduler_name = m.scheduler.type if m.scheduler else None
        self.scheduler_params = dict(m.scheduler.params) if m.scheduler else {}
        self.comms_logger = m.comms_logger
        self.seed = m.seed
        if "bfloat16" in raw and "bf16" not in raw:  # reference alias (runtime/constants.py BFLOAT16_OLD)
            self.model.bf16 = BF16Config(**raw["bfloat16"])
        self.bfloat16_enabled = m.bf16.enabled
        if "use_node_local_storage" in raw and "use_node_local_storage" not in raw.get("checkpoint", {}):
            # legacy root-level spelling of checkpoint.use_node_local_storage
            self.model.checkpoint.use_node_local_storage = bool(raw["use_node_local_storage"])
        self.torch_autocast_enabled = m.torch_autocast.enabled
        self.unknown_keys = self._check_unknown_keys()
        self.grad_accum_dtype = self._grad_accum_dtype()
        self.ignored_knobs = self._check_ignored_knobs()

    def _check_unknown_keys(self):
        """Every key no block defines, as dotted paths. Warns (naming the closest known field) or,
        with ``strict_config`` / SXE_STRICT_CONFIG=1, raises."""
        import difflib
        out = []

        def walk(model, path):
            for k in (getattr(model, "__pydantic_extra__", None) or {}):
                if not path and k in RAW_ROOT_KEYS:
                    continue
                known = list(type(model).model_fields) + [f.alias for f in type(model).model_fields.values()
                                                          if f.alias]
                near = difflib.get_close_matches(k, known, n=1)
                out.append((".".join(path + [k]), near[0] if near else None))
            for name in type(model).model_fields:
                v = getattr(model, name, None)
                if isinstance(v, BaseModel):
                    walk(v, path + [name])
        walk(self.model, [])
        if not out:
            return []
        msg = "; ".join(f"'{k}'" + (f" (did you mean '{n}'?)" if n else "") for k, n in out)
        if self.model.strict_config or os.environ.get("SXE_STRICT_CONFIG", "0") == "1":
            raise ValueError(f"config: unknown keys: {msg}")
        logger.warning(f"config: unknown keys are ignored: {msg}")
        return [k for k, _ in out]

    def _grad_accum_dtype(self):
        """Reference runtime/engine.py:1074-1089 get_data_types: explicit data_types.grad_accum_dtype,
        else fp32 for bf16 without ZeRO, else the model dtype."""
        name = self.model.data_types.grad_accum_dtype
        if name is not None:
            return {"fp32": "fp32", "float32": "fp32", "fp16": "fp16", "float16": "fp16", "bf16": "bf16",
                    "bfloat16": "bf16"}[name]
        if self.bfloat16_enabled and not self.zero_enabled:
            return "fp32"
        return "fp16" if self.fp16_enabled else ("bf16" if self.bfloat16_enabled else "fp32")

    # Reference knobs that are accepted for config compatibility but have no effect here, with the
    # reason. Setting one explicitly logs a warning (never silent); ``ignored_knobs`` lists them.
    IGNORED_ZERO_KNOBS = {
        "sub_group_size": "the fused optimizer step is ONE multi-tensor HIP launch over all fp32 chunks "
                          "(the host tier streams its own fixed-size buffers)",
        "round_robin_gradients": "gradient partitions are flat units reduce-scattered straight into their owner",
        "mics_hierarchical_params_gather": "single-node xGMI: the MiCS shard group is gathered in one step",
        "allgather_bucket_size": "ZeRO-1/2 all-gather one flat unit at a time (units are sized by reduce_bucket_size)",
        "contiguous_gradients": "gradients always land in contiguous flat units",
        "use_multi_rank_bucket_allreduce": "ZeRO-1/2 always use a true reduce-scatter",
        "legacy_stage1": "one ZeRO-1/2 implementation",
        "memory_efficient_linear": "ops/linear.py always writes weight gradients into the ZeRO buffers",
        "pipeline_loading_checkpoint": "checkpoint loading is not pipelined",
    }

    def _check_ignored_knobs(self):
        zc = self.zero_config
        set_ = set(getattr(zc, "model_fields_set", set()))
        out = []
        for k, why in self.IGNORED_ZERO_KNOBS.items():
            if k in set_:
                out.append((f"zero_optimization.{k}", why))
        if self.model.sparse_gradients and zc.stage > 0:
            out.append(("sparse_gradients", "under ZeRO stages 1-3 embedding gradients are reduced densely inside "
                                            "the flat units (same numerics); the sparse all-gather runs at stage 0"))
        neb = self._param_dict.get("nebula")
        if isinstance(neb, dict) and neb.get("enabled"):
            out.append(("nebula", "the Azure Nebula checkpoint service is not available; checkpoints are written by "
                                  "the torch / fast / decoupled engines (checkpoint.writer, checkpoint.async_save)"))
        if self._param_dict.get("mesh_param") is not None:
            out.append(("mesh_param", "a config key has no effect: pass mesh_param=(dp, sp) to initialize(), or set "
                                      "data_parallel_size and sequence_parallel_size"))
        for k, why in out:
            logger.warning(f"config: '{k}' is accepted but has no effect: {why}")
        return out

    def _solve_batch(self):
        m = self.model
        tb, mb, gas = m.train_batch_size, m.train_micro_batch_size_per_gpu, m.gradient_accumulation_steps
        dp = self.dp_world_size
        if m.elasticity.enabled:
            # elastic batch: pick the batch valid for the most GPU counts (reference config.py:870-936)
            from ..elasticity import compute_elastic_config
            el = m.elasticity.model_dump() if hasattr(m.elasticity, "model_dump") else dict(m.elasticity)
            tb, _, mb = compute_elastic_config({"elasticity": el}, world_size=self.world_size, return_microbatch=True)
            if not el.get("ignore_non_elastic_batch_info", False) and m.train_batch_size not in (None, tb):
                logger.warning(f"elasticity overrides train_batch_size {m.train_batch_size} -> {tb}")
            gas = None
        if tb is not None and mb is not None and gas is not None:
            pass
        elif tb is not None and mb is not None:
            gas = tb // (mb * dp)
        elif tb is not None and gas is not None:
            mb = tb // (gas * dp)
        elif mb is not None and gas is not None:
            tb = mb * gas * dp
        elif tb is not None:
            gas = 1
            mb = tb // dp
        elif mb is not None:
            gas = 1
            tb = mb * dp
        else:
            mb, gas = 1, 1
            tb = dp
        if tb != mb * gas * dp or mb < 1 or gas < 1:
            raise ValueError(f"train_batch_size ({tb}) != micro_batch ({mb}) * grad_accum ({gas}) * dp_world ({dp})")
        self.train_batch_size = tb
        self.train_micro_batch_size_per_gpu = mb
        self.gradient_accumulation_steps = gas

    def __getattr__(self, name):
        # fall through to the model for any reference key
        model = self.__dict__.get("model")
        if model is not None and hasattr(model, name):
            return getattr(model, name)
        raise AttributeError(name)

    def to_dict(self):
        return self.model.model_dump(by_alias=False)

    def print(self, name="SXEConfig"):
        logger.info(f"{name}: {json.dumps(self._param_dict, indent=2, default=str)}")


DeepSpeedConfig = SXEConfig
