"""``FP16_UnfusedOptimizer`` (reference runtime/fp16/unfused_optimizer.py:24): per-parameter fp32
masters for layer-wise optimizers (LAMB). Here: the data-parallel flat-unit optimizer with one
bucket per parameter, so the layer-wise optimizer sees per-parameter segments (ops/optim.py
FusedLamb.set_segments) exactly like the reference's unfused per-tensor masters; static or dynamic
loss scaling with the overflow check on the device."""


def FP16_UnfusedOptimizer(init_optimizer, deepspeed=None, static_loss_scale=1.0, dynamic_loss_scale=False,
                          dynamic_loss_args=None, verbose=True, mpu=None, clip_grad=0.0, fused_lamb_legacy=False):
    from ..zero.stage0 import DataParallelOptimizer
    from .fused_optimizer import _scaler
    return DataParallelOptimizer(init_optimizer,
                                 loss_scaler=_scaler(static_loss_scale, dynamic_loss_scale, 2**32, dynamic_loss_args),
                                 clip_grad=clip_grad, bucket_size=1)
