"""Learning-rate schedules (parity: reference runtime/lr_schedules.py -- LRRangeTest :273,
OneCycle :371, WarmupLR :633, WarmupDecayLR :726, WarmupCosineLR :777). Same names, config keys
and step semantics (`step()` once per optimizer step, `last_batch_iteration` state)."""
import math

LR_RANGE_TEST = "LRRangeTest"
ONE_CYCLE = "OneCycle"
WARMUP_LR = "WarmupLR"
WARMUP_DECAY_LR = "WarmupDecayLR"
WARMUP_COSINE_LR = "WarmupCosineLR"
VALID_LR_SCHEDULES = [LR_RANGE_TEST, ONE_CYCLE, WARMUP_LR, WARMUP_DECAY_LR, WARMUP_COSINE_LR]
WARMUP_LOG_RATE, WARMUP_LINEAR_RATE = "log", "linear"


def _groups(optimizer):
    return optimizer.param_groups


def _per_group(optimizer, v):
    n = len(_groups(optimizer))
    if isinstance(v, (list, tuple)):
        if len(v) != n:
            raise ValueError(f"expected {n} values, got {len(v)}")
        return list(v)
    return [v] * n


def _set_lrs(optimizer, lrs):
    # ``lr_mult``: per-group learning-rate multiplier that schedules must keep (muP width scaling,
    # ops/optim.py mup_param_groups)
    for g, lr in zip(_groups(optimizer), lrs):
        g["lr"] = lr * g.get("lr_mult", 1.0)
    return [g["lr"] for g in _groups(optimizer)]


class _Sched:
    last_batch_iteration = -1

    def get_last_lr(self):
        return self._last_lr

    def step(self, last_batch_iteration=None):
        self.last_batch_iteration = (self.last_batch_iteration + 1) if last_batch_iteration is None else last_batch_iteration
        self._last_lr = _set_lrs(self.optimizer, self.get_lr())

    def state_dict(self):
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd):
        self.last_batch_iteration = sd["last_batch_iteration"]


class WarmupLR(_Sched):
    def __init__(self, optimizer, warmup_min_lr=0.0, warmup_max_lr=None, warmup_num_steps=1000,
                 warmup_type=WARMUP_LOG_RATE, last_batch_iteration=-1):
        self.optimizer = optimizer
        if warmup_max_lr is None:
            warmup_max_lr = [g["lr"] / g.get("lr_mult", 1.0) for g in _groups(optimizer)]
        self.min_lrs = _per_group(optimizer, warmup_min_lr)
        self.max_lrs = _per_group(optimizer, warmup_max_lr)
        self.warmup_num_steps = max(2, int(warmup_num_steps))
        self.warmup_type = warmup_type if warmup_type in (WARMUP_LOG_RATE, WARMUP_LINEAR_RATE) else WARMUP_LOG_RATE
        self.last_batch_iteration = last_batch_iteration
        if last_batch_iteration == -1:
            self._last_lr = _set_lrs(optimizer, self.get_lr())

    def _warm(self):
        it = self.last_batch_iteration
        if self.warmup_type == WARMUP_LOG_RATE:
            return math.log(it + 1) / math.log(self.warmup_num_steps)
        return it / self.warmup_num_steps

    def _gamma(self):
        return self._warm() if self.last_batch_iteration < self.warmup_num_steps else 1.0

    def get_lr(self):
        if self.last_batch_iteration < 0:
            return list(self.min_lrs)
        g = self._gamma()
        return [lo + (hi - lo) * g for lo, hi in zip(self.min_lrs, self.max_lrs)]


class WarmupDecayLR(WarmupLR):
    def __init__(self, optimizer, total_num_steps, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 warmup_type=WARMUP_LOG_RATE, last_batch_iteration=-1):
        self.total_num_steps = total_num_steps
        super().__init__(optimizer, warmup_min_lr, warmup_max_lr, warmup_num_steps, warmup_type, last_batch_iteration)

    def _gamma(self):
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            return self._warm()
        return max(0.0, float(self.total_num_steps - it) / float(max(1.0, self.total_num_steps - self.warmup_num_steps)))


class WarmupCosineLR(_Sched):
    def __init__(self, optimizer, total_num_steps, warmup_min_ratio=0.0, warmup_num_steps=1000, cos_min_ratio=0.0001,
                 warmup_type=WARMUP_LOG_RATE, last_batch_iteration=-1):
        self.optimizer = optimizer
        self.total_num_steps = total_num_steps
        self.warmup_min_ratio = warmup_min_ratio
        self.warmup_num_steps = max(2, int(warmup_num_steps))
        self.cos_min_ratio = cos_min_ratio
        self.warmup_type = warmup_type
        self.last_batch_iteration = last_batch_iteration
        self.org_lrs = [g["lr"] / g.get("lr_mult", 1.0) for g in _groups(optimizer)]
        if last_batch_iteration == -1:
            self._last_lr = _set_lrs(optimizer, self.get_lr())

    def get_lr_ratio(self):
        it = self.last_batch_iteration
        if it < 0:
            return 0.0
        if it < self.warmup_num_steps:
            if self.warmup_type == WARMUP_LOG_RATE:
                r = math.log(it + 1) / math.log(self.warmup_num_steps)
            else:
                r = it / self.warmup_num_steps
            return self.warmup_min_ratio + (1.0 - self.warmup_min_ratio) * r
        progress = (it - self.warmup_num_steps) / max(1, self.total_num_steps - self.warmup_num_steps)
        progress = min(1.0, progress)
        cos = 0.5 * (1.0 + math.cos(math.pi * progress))
        return self.cos_min_ratio + (1.0 - self.cos_min_ratio) * cos

    def get_lr(self):
        r = self.get_lr_ratio()
        return [lr * r for lr in self.org_lrs]


class LRRangeTest(_Sched):
    def __init__(self, optimizer, lr_range_test_min_lr=1e-3, lr_range_test_step_size=2000,
                 lr_range_test_step_rate=1.0, lr_range_test_staircase=False, last_batch_iteration=-1):
        self.optimizer = optimizer
        self.min_lr = _per_group(optimizer, lr_range_test_min_lr)
        self.step_size = lr_range_test_step_size
        self.step_rate = lr_range_test_step_rate
        self.staircase = lr_range_test_staircase
        self.last_batch_iteration = last_batch_iteration
        if last_batch_iteration == -1:
            self._last_lr = _set_lrs(optimizer, self.get_lr())

    def get_lr(self):
        it = max(0, self.last_batch_iteration + 1)
        x = it / self.step_size
        if self.staircase:
            x = math.floor(x)
        f = 1 + self.step_rate * x
        return [lr * f for lr in self.min_lr]


class OneCycle(_Sched):
    def __init__(self, optimizer, cycle_min_lr, cycle_max_lr, decay_lr_rate=0.0, cycle_first_step_size=2000,
                 cycle_second_step_size=None, cycle_first_stair_count=0, cycle_second_stair_count=None,
                 decay_step_size=0, cycle_momentum=True, cycle_min_mom=0.8, cycle_max_mom=0.9, decay_mom_rate=0.0,
                 last_batch_iteration=-1):
        self.optimizer = optimizer
        self.min_lrs = _per_group(optimizer, cycle_min_lr)
        self.max_lrs = _per_group(optimizer, cycle_max_lr)
        self.decay_lr_rate = decay_lr_rate
        self.first = float(cycle_first_step_size)
        self.second = float(cycle_second_step_size if cycle_second_step_size is not None else cycle_first_step_size)
        self.total = self.first + self.second
        self.decay_step_size = decay_step_size
        self.cycle_momentum = cycle_momentum
        self.min_mom, self.max_mom, self.decay_mom_rate = cycle_min_mom, cycle_max_mom, decay_mom_rate
        self.last_batch_iteration = last_batch_iteration
        if last_batch_iteration == -1:
            self._last_lr = _set_lrs(optimizer, self.get_lr())

    def _cycle_frac(self, it):
        if it <= self.first:
            return it / self.first
        return max(0.0, 1.0 - (it - self.first) / self.second)

    def get_lr(self):
        it = max(0, self.last_batch_iteration)
        if it < self.total:
            f = self._cycle_frac(it)
            return [lo + (hi - lo) * f for lo, hi in zip(self.min_lrs, self.max_lrs)]
        decay_steps = (it - self.total) / self.decay_step_size if self.decay_step_size else 0
        factor = 1.0 / (1.0 + self.decay_lr_rate * decay_steps)
        return [lo * factor for lo in self.min_lrs]

    def get_mom(self):
        it = max(0, self.last_batch_iteration)
        if it < self.total:
            f = self._cycle_frac(it)
            return self.max_mom - (self.max_mom - self.min_mom) * f
        return self.max_mom

    def step(self, last_batch_iteration=None):
        super().step(last_batch_iteration)
        if self.cycle_momentum:
            m = self.get_mom()
            for g in _groups(self.optimizer):
                if "betas" in g:
                    g["betas"] = (m, g["betas"][1])
                elif "momentum" in g:
                    g["momentum"] = m


def build_scheduler(name, optimizer, params):
    table = {WARMUP_LR: WarmupLR, WARMUP_DECAY_LR: WarmupDecayLR, WARMUP_COSINE_LR: WarmupCosineLR,
             LR_RANGE_TEST: LRRangeTest, ONE_CYCLE: OneCycle}
    if name not in table:
        raise ValueError(f"unknown scheduler {name}; valid: {VALID_LR_SCHEDULES}")
    return table[name](optimizer, **params)
