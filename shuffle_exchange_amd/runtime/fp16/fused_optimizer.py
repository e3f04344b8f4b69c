"""FP16 / BF16 mixed-precision optimizer wrappers without ZeRO partitioning.

Parity: reference runtime/fp16/fused_optimizer.py:33 ``FP16_Optimizer`` (flat fp32 masters, one
fused step, static/dynamic loss scaling), runtime/fp16/unfused_optimizer.py:24
``FP16_UnfusedOptimizer`` (per-parameter masters, for LAMB-style layer-wise optimizers) and
runtime/bf16_optimizer.py:35 ``BF16_Optimizer`` (bf16 params, fp32 gradient accumulation,
ZeRO-1-like partitioned fp32 state). All three map onto this framework's flat-unit optimizers
(runtime/zero/stage0.py, stage12.py): masters live in one fp32 buffer per parameter group, the
update is one multi-tensor HIP launch that writes the 16-bit copy back, the overflow check and the
loss-scale update stay on the device. The constructors accept the reference's keyword arguments.
"""
import torch

from .loss_scaler import DynamicLossScaler, LossScaler


def _scaler(static_loss_scale, dynamic_loss_scale, initial_dynamic_scale, dynamic_loss_args):
    if dynamic_loss_scale:
        a = dict(dynamic_loss_args or {})
        return DynamicLossScaler(init_scale=a.get("init_scale", initial_dynamic_scale),
                                 scale_window=a.get("scale_window", 1000), min_scale=a.get("min_scale", 1.0),
                                 delayed_shift=a.get("delayed_shift", 1),
                                 consecutive_hysteresis=a.get("consecutive_hysteresis", False))
    return LossScaler(static_loss_scale)


def FP16_Optimizer(init_optimizer, deepspeed=None, static_loss_scale=1.0, dynamic_loss_scale=False,
                   initial_dynamic_scale=2**32, dynamic_loss_args=None, verbose=True, mpu=None, clip_grad=0.0,
                   fused_adam_legacy=False, has_moe_layers=False, timers=None):
    from ..zero.stage0 import DataParallelOptimizer
    return DataParallelOptimizer(init_optimizer,
                                 loss_scaler=_scaler(static_loss_scale, dynamic_loss_scale, initial_dynamic_scale,
                                                     dynamic_loss_args), clip_grad=clip_grad)


def FP16_UnfusedOptimizer(init_optimizer, deepspeed=None, static_loss_scale=1.0, dynamic_loss_scale=False,
                          dynamic_loss_args=None, verbose=True, mpu=None, clip_grad=0.0, fused_lamb_legacy=False):
    # one bucket per parameter: layer-wise optimizers see per-parameter segments (ops/optim.py
    # FusedLamb.set_segments) exactly like the reference's unfused per-tensor masters
    from ..zero.stage0 import DataParallelOptimizer
    return DataParallelOptimizer(init_optimizer,
                                 loss_scaler=_scaler(static_loss_scale, dynamic_loss_scale, 2**32, dynamic_loss_args),
                                 clip_grad=clip_grad, bucket_size=1)


def BF16_Optimizer(init_optimizer, param_names=None, bfloat16_config=None, mpu=None, clip_grad=0.0, norm_type=2,
                   allgather_bucket_size=5000000000, dp_process_group=None, timers=None, grad_acc_dtype=None,
                   graph_harvesting=False, immediate_grad_update=False, has_moe_layers=False):
    from ...parallel import groups
    from ..zero.stage12 import ZeroStage12Optimizer
    return ZeroStage12Optimizer(init_optimizer, stage=1, loss_scaler=LossScaler(1.0), clip_grad=clip_grad,
                                dp_ranks=groups.group_ranks("seq_data"), dp_group=dp_process_group,
                                reduce_bucket_size=min(int(allgather_bucket_size), 500_000_000))


__all__ = ["FP16_Optimizer", "FP16_UnfusedOptimizer", "BF16_Optimizer", "torch"]
