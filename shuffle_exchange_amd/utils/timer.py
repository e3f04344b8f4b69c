"""Timers (parity: reference deepspeed/utils/timer.py:44 SynchronizedWallClockTimer, :199
ThroughputTimer). Adds what the reference lacks: tokens/s and model TFLOPs/GPU."""
import time

import torch

from ..accelerator import get_accelerator
from .logging import log_dist


class _Timer:
    def __init__(self, name, use_events):
        self.name = name
        self.use_events = use_events
        self.started = False
        self.elapsed_ = 0.0
        self.count = 0
        self._t0 = None
        self._events = []

    def start(self):
        if self.started:
            return
        if self.use_events:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._t0 = e
        else:
            self._t0 = time.perf_counter()
        self.started = True

    def stop(self, reset=False, record=False):
        if not self.started:
            return
        if self.use_events:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append((self._t0, e))
        else:
            self.elapsed_ += time.perf_counter() - self._t0
        self.count += 1
        self.started = False

    def _drain(self):
        if self._events:
            self._events[-1][1].synchronize()
            for a, b in self._events:
                self.elapsed_ += a.elapsed_time(b) / 1000.0
            self._events = []

    def reset(self):
        self._drain()
        self.elapsed_ = 0.0
        self.count = 0
        self.started = False

    def elapsed(self, reset=True):
        was = self.started
        if was:
            self.stop()
        self._drain()
        v = self.elapsed_
        if reset:
            self.elapsed_ = 0.0
            self.count = 0
        if was:
            self.start()
        return v

    def mean(self):
        self._drain()
        return self.elapsed_ / max(1, self.count)


class SynchronizedWallClockTimer:
    """Named timers backed by HIP events (no host sync until read)."""

    def __init__(self):
        self.timers = {}
        self.use_events = get_accelerator().gpu

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name, self.use_events)
        return self.timers[name]

    def get_timers(self):
        return self.timers

    def log(self, names, normalizer=1.0, reset=True, memory_breakdown=False, ranks=None):
        parts = []
        for n in names:
            if n in self.timers:
                parts.append(f"{n}: {self.timers[n].elapsed(reset=reset) * 1000.0 / normalizer:.2f}")
        if parts:
            log_dist("time (ms) | " + " | ".join(parts), ranks=ranks or [0])

    def get_mean(self, names, normalizer=1.0, reset=True):
        out = {}
        for n in names:
            if n in self.timers:
                out[n] = self.timers[n].mean() * 1000.0 / normalizer
                if reset:
                    self.timers[n].reset()
        return out


class NoopTimer:
    class _T:
        def start(self):
            pass

        def stop(self, **kw):
            pass

        def reset(self):
            pass

        def elapsed(self, **kw):
            return 0.0

        def mean(self):
            return 0.0

    def __init__(self):
        self._t = NoopTimer._T()

    def __call__(self, name):
        return self._t

    def get_timers(self):
        return {}

    def log(self, *a, **k):
        pass

    def get_mean(self, *a, **k):
        return {}


class ThroughputTimer:
    """samples/s, tokens/s and model TFLOPs per GPU over the global steps since ``start_step``
    (reference utils/timer.py:199). Each micro-step's [forward .. step] segment is bracketed by
    HIP events: nothing synchronises the host until a report is due (the reference synchronises
    the device at every start/stop)."""

    def __init__(self, batch_size, seq_len=None, flops_per_sample=None, start_step=2, steps_per_output=50,
                 monitor_memory=False, logging_fn=None):
        self.batch_size = batch_size
        self.seq_len = seq_len
        self.flops_per_sample = flops_per_sample
        self.start_step = start_step
        self.steps_per_output = steps_per_output
        self.logging = logging_fn or (lambda m: log_dist(m, ranks=[0]))
        self.monitor_memory = monitor_memory
        self.use_events = get_accelerator().gpu
        self.global_step_count = 0
        self.micro_step_count = 0
        self.total_elapsed_time = 0.0
        self.step_elapsed_time = 0.0
        self._t = None
        self._pending = []
        self.started = False
        self.last_report = None

    def update_epoch_count(self):
        pass

    def _now(self):
        if self.use_events:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def start(self):
        if self.started:
            return
        self.started = True
        if self.global_step_count >= self.start_step:
            self._t = self._now()

    def _drain(self):
        if not self._pending:
            return
        if self.use_events:
            self._pending[-1][1].synchronize()
            dt = sum(a.elapsed_time(b) for a, b in self._pending) / 1000.0
        else:
            dt = sum(b - a for a, b in self._pending)
        self._pending = []
        self.total_elapsed_time += dt
        self.step_elapsed_time += dt

    def stop(self, global_step=False, report_speed=True):
        if not self.started:
            return None
        self.started = False
        self.micro_step_count += 1
        if global_step:
            self.global_step_count += 1
        if self._t is not None:
            self._pending.append((self._t, self._now()))
            self._t = None
        if global_step and report_speed and self.steps_per_output and \
                self.global_step_count % self.steps_per_output == 0 and self._timed_steps() > 0:
            self._drain()
            rep = {"samples_per_sec": self.avg_samples_per_sec()}
            msg = f"step={self.global_step_count} samples/s={rep['samples_per_sec']:.2f}"
            if self.seq_len:
                rep["tokens_per_sec"] = self.avg_tokens_per_sec()
                msg += f" tokens/s={rep['tokens_per_sec']:.1f}"
            if self.flops_per_sample:
                rep["tflops"] = self.avg_tflops()
                msg += f" TFLOPs/GPU={rep['tflops']:.1f}"
            if self.monitor_memory:
                msg += f" mem_alloc_GB={get_accelerator().memory_allocated() / 2**30:.2f}"
            self.logging(msg)
            self.step_elapsed_time = 0.0
            self.last_report = rep
            return rep
        return None

    def _timed_steps(self):
        return max(0, self.global_step_count - self.start_step)

    def avg_samples_per_sec(self):
        self._drain()
        n = self._timed_steps()
        return (n * self.batch_size / self.total_elapsed_time) if n > 0 and self.total_elapsed_time > 0 else 0.0

    def avg_tokens_per_sec(self):
        return self.avg_samples_per_sec() * (self.seq_len or 1)

    def avg_tflops(self):
        """Model TFLOP/s per GPU (``flops_per_sample`` is the whole-model cost of one sample;
        ``batch_size`` is the global batch, so divide by the data-parallel world)."""
        ws = max(1, getattr(self, "world_size", 1))
        return self.avg_samples_per_sec() * (self.flops_per_sample or 0) / ws / 1e12
