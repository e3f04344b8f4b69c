"""Autotuner: search ZeRO stage x micro-batch size (x any other config knob) for the best training
throughput with short profiled runs.

Parity: reference autotuning/autotuner.py (``Autotuner`` :42: model-info profiling, memory-based
pruning of infeasible stages, per-stage micro-batch search, tuners in autotuning/tuner/ --
``GridSearchTuner``, ``RandomTuner``, ``ModelBasedTuner`` (XGBoost cost model) --, experiment
scheduling autotuning/scheduler.py:32, results under ``autotuning_results`` / ``autotuning_exps``,
and the engine side that measures ``start_profile_step .. end_profile_step`` and writes the metric).

Differences: experiments are either callables (in-process, for tests / notebooks) or launched as
subprocesses of the user script with a generated config; the model-based tuner fits a small
least-squares cost model over the features (log2 mbs, stage one-hot) instead of XGBoost (not
available offline); memory pruning uses the per-stage model-state formula for 288 GB MI355X HBM.
"""
import itertools
import json
import math
import os
import random
import subprocess
import sys
import time

import numpy as np

HBM_BYTES = 288 * 2**30


def model_state_bytes(num_params, stage, dp, bit16=2, master=4, optim=8):
    """Bytes per GPU for params + grads + optimizer states under ZeRO-`stage` (no activations)."""
    p = num_params
    if stage == 0:
        return p * (bit16 + 4 + master + optim)
    if stage == 1:
        return p * (bit16 + 4) + p * (master + optim) / dp
    if stage == 2:
        return p * bit16 + p * (4 + master + optim) / dp
    return p * (bit16 + 4 + master + optim) / dp


class Experiment:
    def __init__(self, name, overrides):
        self.name = name
        self.overrides = overrides
        self.metric = None
        self.error = None

    def __repr__(self):
        return f"Experiment({self.name}, metric={self.metric})"


class BaseTuner:
    def __init__(self, experiments, run_fn, metric="throughput"):
        self.all = list(experiments)
        self.run_fn = run_fn
        self.metric = metric
        self.best = None

    def _evaluate(self, exp):
        try:
            exp.metric = self.run_fn(exp)
        except Exception as e:  # an OOM / failing config is just a bad point
            exp.error = repr(e)
            exp.metric = None
        if exp.metric is not None and (self.best is None or exp.metric > self.best.metric):
            self.best = exp
        return exp.metric

    def next_batch(self, n):
        raise NotImplementedError

    def tune(self, n_trials=None, early_stopping=None):
        n_trials = n_trials or len(self.all)
        done, since_best = 0, 0
        while done < n_trials:
            batch = self.next_batch(1)
            if not batch:
                break
            for e in batch:
                prev = self.best
                self._evaluate(e)
                done += 1
                since_best = 0 if self.best is not prev else since_best + 1
            if early_stopping and since_best >= early_stopping:
                break
        return self.best


class GridSearchTuner(BaseTuner):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._queue = list(self.all)

    def next_batch(self, n):
        out, self._queue = self._queue[:n], self._queue[n:]
        return out


class RandomTuner(GridSearchTuner):
    def __init__(self, *a, seed=1234, **k):
        super().__init__(*a, **k)
        random.Random(seed).shuffle(self._queue)


class ModelBasedTuner(BaseTuner):
    """Evaluate a few random points, then always the point the fitted cost model ranks best."""

    def __init__(self, *a, warmup=3, seed=1234, **k):
        super().__init__(*a, **k)
        self._left = list(self.all)
        random.Random(seed).shuffle(self._left)
        self.warmup = warmup
        self._seen = []

    @staticmethod
    def _feat(e):
        o = e.overrides
        mbs = o.get("train_micro_batch_size_per_gpu", 1)
        st = o.get("zero_optimization", {}).get("stage", 0)
        return [1.0, math.log2(max(1, mbs)), math.log2(max(1, mbs)) ** 2] + [float(st == s) for s in range(4)]

    def next_batch(self, n):
        if not self._left:
            return []
        scored = [e for e in self._seen if e.metric is not None]
        if len(scored) < self.warmup:
            pick = self._left.pop()
        else:
            X = np.array([self._feat(e) for e in scored])
            y = np.array([e.metric for e in scored])
            w, *_ = np.linalg.lstsq(X, y, rcond=None)
            preds = [float(np.dot(self._feat(e), w)) for e in self._left]
            pick = self._left.pop(int(np.argmax(preds)))
        self._seen.append(pick)
        return [pick]


TUNERS = {"gridsearch": GridSearchTuner, "random": RandomTuner, "model_based": ModelBasedTuner}


def _deep_update(d, u):
    out = dict(d)
    for k, v in u.items():
        out[k] = _deep_update(out.get(k, {}), v) if isinstance(v, dict) else v
    return out


class Autotuner:
    def __init__(self, base_config, num_params=None, world_size=1, results_dir="autotuning_results",
                 exps_dir="autotuning_exps", tuner_type="gridsearch", tuner_num_trials=50, tuner_early_stopping=5,
                 micro_batch_sizes=None, stages=(0, 1, 2, 3), hbm_bytes=HBM_BYTES, metric="throughput"):
        self.base = dict(base_config)
        self.num_params = num_params
        self.world = world_size
        self.results_dir, self.exps_dir = results_dir, exps_dir
        self.tuner_type = tuner_type
        self.trials, self.early = tuner_num_trials, tuner_early_stopping
        self.mbs = list(micro_batch_sizes or [1, 2, 4, 8, 16])
        self.stages = list(stages)
        self.hbm = hbm_bytes
        self.metric = metric
        self.records = []

    def feasible_stages(self):
        if not self.num_params:
            return self.stages
        return [s for s in self.stages if model_state_bytes(self.num_params, s, self.world) < 0.9 * self.hbm]

    def experiments(self):
        exps = []
        for st, mb in itertools.product(self.feasible_stages(), self.mbs):
            ov = {"zero_optimization": {"stage": st}, "train_micro_batch_size_per_gpu": mb}
            exps.append(Experiment(f"z{st}_mbs{mb}", ov))
        return exps

    def tune(self, run_fn):
        """run_fn(config_dict) -> metric (higher is better) or raises."""
        def run(exp):
            cfg = _deep_update(self.base, exp.overrides)
            cfg.pop("train_batch_size", None)
            t0 = time.time()
            m = run_fn(cfg)
            self.records.append({"name": exp.name, "config": exp.overrides, "metric": m, "secs": time.time() - t0})
            return m

        tuner = TUNERS[self.tuner_type](self.experiments(), run, metric=self.metric)
        best = tuner.tune(self.trials, self.early)
        self.best = best
        os.makedirs(self.results_dir, exist_ok=True)
        with open(os.path.join(self.results_dir, "summary.json"), "w") as f:
            json.dump({"best": best.name if best else None, "best_metric": best.metric if best else None,
                       "best_config": _deep_update(self.base, best.overrides) if best else None,
                       "experiments": self.records}, f, indent=2)
        return best

    def best_config(self):
        return _deep_update(self.base, self.best.overrides) if getattr(self, "best", None) else None


def subprocess_runner(user_script, user_args=(), exps_dir="autotuning_exps", nproc=1, timeout=1800,
                      start_step=3, end_step=5):
    """run_fn that launches the user script with a generated config and reads the metric file the
    engine writes (``autotuning.metric_path``)."""
    def run(cfg):
        os.makedirs(exps_dir, exist_ok=True)
        tag = f"exp_{len(os.listdir(exps_dir))}"
        mpath = os.path.abspath(os.path.join(exps_dir, tag + "_metric.json"))
        cfg = _deep_update(cfg, {"autotuning": {"enabled": True, "metric_path": mpath, "start_profile_step": start_step,
                                                "end_profile_step": end_step}})
        cpath = os.path.join(exps_dir, tag + "_config.json")
        with open(cpath, "w") as f:
            json.dump(cfg, f)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(29700 + random.randint(0, 200)), user_script,
               "--deepspeed_config", cpath] + list(user_args)
        subprocess.run(cmd, timeout=timeout, check=False)
        if not os.path.exists(mpath):
            raise RuntimeError(f"experiment {tag} produced no metric")
        with open(mpath) as f:
            return json.load(f)["throughput"]
    return run
