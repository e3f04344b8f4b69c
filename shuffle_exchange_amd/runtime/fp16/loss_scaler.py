"""Static and dynamic loss scaling (parity: reference runtime/fp16/loss_scaler.py:69 LossScaler,
:93 DynamicLossScaler, :211 CreateLossScaler).

Checkpoints store ``state_dict()`` (plain numbers) instead of the pickled scaler object the
reference writes, so they load with ``torch.load(weights_only=True)``.
"""
import torch

INITIAL_LOSS_SCALE = "init_scale"
SCALE_WINDOW = "scale_window"
DELAYED_SHIFT = "delayed_shift"
CONSECUTIVE_HYSTERESIS = "consecutive_hysteresis"
MIN_LOSS_SCALE = "min_scale"


class LossScalerBase:
    def __init__(self, cur_scale):
        self.cur_scale = cur_scale
        self.dynamic = False

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def update_scale(self, overflow):
        pass

    def backward(self, loss, retain_graph=False):
        (loss * self.loss_scale).backward(retain_graph=retain_graph)

    def state_dict(self):
        return {"cur_scale": self.cur_scale, "dynamic": self.dynamic}

    def load_state_dict(self, sd):
        self.cur_scale = sd["cur_scale"]


class LossScaler(LossScalerBase):
    def __init__(self, scale=1):
        super().__init__(scale)

    def has_overflow(self, params):
        return False


class DynamicLossScaler(LossScalerBase):
    def __init__(self, init_scale=2**32, scale_factor=2.0, scale_window=1000, min_scale=1, delayed_shift=1,
                 consecutive_hysteresis=False, raise_error_at_min_scale=True, dtype=torch.half):
        super().__init__(init_scale)
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis
        self.raise_error_at_min_scale = raise_error_at_min_scale
        self.dynamic = True
        self.dtype = dtype

    def update_scale(self, overflow):
        if overflow:
            if self.delayed_shift == 1 or self.cur_hysteresis == 1:
                if self.cur_scale == self.min_scale and self.raise_error_at_min_scale:
                    raise RuntimeError("Current loss scale already at minimum - cannot decrease scale anymore.")
                self.cur_scale = max(self.cur_scale / self.scale_factor, self.min_scale)
            else:
                self.cur_hysteresis -= 1
            self.last_overflow_iter = self.cur_iter
        else:
            if self.consecutive_hysteresis:
                self.cur_hysteresis = self.delayed_shift
            if (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
                if not self.consecutive_hysteresis:
                    self.cur_hysteresis = self.delayed_shift
                self.cur_scale *= self.scale_factor
        self.cur_iter += 1

    def state_dict(self):
        d = super().state_dict()
        d.update(cur_iter=self.cur_iter, last_overflow_iter=self.last_overflow_iter,
                 cur_hysteresis=self.cur_hysteresis)
        return d

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        self.cur_iter = sd.get("cur_iter", 0)
        self.last_overflow_iter = sd.get("last_overflow_iter", -1)
        self.cur_hysteresis = sd.get("cur_hysteresis", self.delayed_shift)


def CreateLossScaler(dtype, static_loss_scale, dynamic_scaling, dynamic_loss_args):
    if dtype == torch.half and dynamic_scaling:
        return DynamicLossScaler(dtype=dtype, **(dynamic_loss_args or {}))
    scale = static_loss_scale if dtype == torch.half else 1.0
    return LossScaler(scale=scale)


def make_scaler(cfg, dtype):
    """From an FP16Config: loss_scale == 0 -> dynamic."""
    if dtype != torch.float16:
        return LossScaler(1.0)
    if cfg.loss_scale and cfg.loss_scale > 0:
        return LossScaler(cfg.loss_scale)
    return DynamicLossScaler(init_scale=2**cfg.initial_scale_power, scale_window=cfg.loss_scale_window,
                             min_scale=cfg.min_loss_scale, delayed_shift=cfg.hysteresis,
                             consecutive_hysteresis=cfg.consecutive_hysteresis)
