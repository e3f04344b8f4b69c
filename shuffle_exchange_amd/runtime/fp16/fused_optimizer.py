"""FP16 / BF16 mixed-precision optimizer wrappers without ZeRO partitioning.

Parity: reference runtime/fp16/fused_optimizer.py:33 ``FP16_Optimizer`` (flat fp32 masters, one
fused step, static/dynamic loss scaling), runtime/fp16/unfused_optimizer.py:24
``FP16_UnfusedOptimizer`` (unfused_optimizer.py here) and runtime/bf16_optimizer.py:35
``BF16_Optimizer`` (runtime/bf16_optimizer.py here). All three map onto this framework's flat-unit optimizers
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


def BF16_Optimizer(*args, **kwargs):
    from ..bf16_optimizer import BF16_Optimizer as _B
    return _B(*args, **kwargs)


from .unfused_optimizer import FP16_UnfusedOptimizer  # noqa: E402


__all__ = ["FP16_Optimizer", "FP16_UnfusedOptimizer", "BF16_Optimizer", "torch"]
