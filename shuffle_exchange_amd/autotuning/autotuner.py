"""Autotuner: search ZeRO stage x micro-batch size (x any other config knob) for the best training
throughput with short profiled runs.

Parity: reference autotuning/autotuner.py (``Autotuner`` :42: model-info profiling, memory-based
pruning of infeasible stages, per-stage micro-batch search, tuners in autotuning/tuner/ --
``GridSearchTuner``, ``RandomTuner``, ``ModelBasedTuner`` (XGBoost cost model) --, experiment
scheduling autotuning/scheduler.py:32, results under ``autotuning_results`` / ``autotuning_exps``,
and the engine side that measures ``start_profile_step .. end_profile_step`` and writes the metric).

Here: experiments are either callables (in-process, for tests / notebooks) or run by
scheduler.ResourceManager (each experiment a process group on its own devices, several at once
when the node has the GPUs); the profiling experiment reports model info from the engine, which
sizes the micro-batch candidates against 288 GB of MI355X HBM; the model-based tuner fits a small
least-squares cost model over (log2 mbs, stage one-hot) instead of XGBoost (not available offline).
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
        if exp.metric is not None and (self.best is None or (exp.metric < self.best.metric if self.metric == "latency"
                                                              else exp.metric > self.best.metric)):
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
    """Evaluate ``warmup`` random points, then mostly the point the refit cost model ranks best,
    with a ``random_ratio`` share of random exploration (reference autotuning/tuner/
    model_based_tuner.py: XGBoost cost model over the flattened numeric config values, 0.2 random
    exploration). The cost model is autotuning/cost_model.py (boosted regression trees)."""

    def __init__(self, *a, warmup=3, seed=1234, random_ratio=0.2, cost_model="gbt", **k):
        super().__init__(*a, **k)
        from .cost_model import ConfigFeaturizer, CostModel
        self._rng = random.Random(seed)
        self._left = list(self.all)
        self._rng.shuffle(self._left)
        self.warmup, self.random_ratio = warmup, random_ratio
        self._seen = []
        self._feat = ConfigFeaturizer([e.overrides for e in self.all])
        self.model = CostModel(cost_model, seed=seed)
        self.lower_is_better = self.metric == "latency"

    def next_batch(self, n):
        if not self._left:
            return []
        scored = [e for e in self._seen if e.metric is not None]
        if len(scored) < self.warmup or self._rng.random() < self.random_ratio:
            pick = self._left.pop()
        else:
            X = [self._feat(e.overrides) for e in scored]
            y = [e.metric for e in scored]
            preds = self.model.fit(X, y).predict([self._feat(e.overrides) for e in self._left])
            i = int(np.argmin(preds) if self.lower_is_better else np.argmax(preds))
            pick = self._left.pop(i)
        self._seen.append(pick)
        return [pick]


TUNERS = {"gridsearch": GridSearchTuner, "random": RandomTuner, "model_based": ModelBasedTuner}


def _deep_update(d, u):
    out = dict(d)
    for k, v in u.items():
        out[k] = _deep_update(out.get(k, {}), v) if isinstance(v, dict) else v
    return out


def _set_path(cfg, dotted, value):
    d = cfg
    keys = dotted.split(".")
    for k in keys[:-1]:
        d = d.setdefault(k, {})
    d[keys[-1]] = value


class Autotuner:
    """Search micro-batch size x ZeRO stage (x each stage's tuning space) for the best metric.

    Flow (reference autotuner.py ``tune`` :410-560):
      1. model info -- from ``autotuning.model_info`` or a profiling experiment whose engine writes
         ``num_params`` / ``activation_mem_per_gpu`` (runtime/engine.py ``_autotuning_probe``);
      2. prune ZeRO stages whose model states cannot fit 90 % of HBM (288 GB per MI355X);
      3. per stage, the largest micro-batch size the memory estimate allows (capped by
         ``max_train_micro_batch_size_per_gpu`` / ``max_train_batch_size``) and
         ``num_tuning_micro_batch_sizes`` candidates between the min and that max, searched by the
         tuner; a stage whose best is < 90 % of the best so far stops the climb to higher stages;
      4. ``fast = False``: the best micro-batch size of each stage is crossed with the stage's tuning
         space (config.DEFAULT_TUNING_SPACE or ``tuning_space``);
      5. results: ``summary.json``, ``ds_config_optimal.json`` and ``cmd_optimal.txt`` in
         ``results_dir``.
    ``run_fn(config) -> metric`` (in process) or a scheduler.ResourceManager runs the experiments."""

    def __init__(self, base_config, num_params=None, world_size=1, results_dir=None, exps_dir=None,
                 tuner_type=None, tuner_num_trials=None, tuner_early_stopping=-1, micro_batch_sizes=None,
                 stages=None, hbm_bytes=HBM_BYTES, metric=None, tuning_space=None, fast=None):
        from .config import AutotuningConfig
        self.base = dict(base_config)
        self.at = AutotuningConfig.from_dict(self.base.get("autotuning", {}))
        at = self.at
        self.num_params = num_params or at.model_info.get("num_params")
        self.model_info = dict(at.model_info)
        if num_params:
            self.model_info["num_params"] = num_params
        self.world = world_size
        self.results_dir = results_dir or at.results_dir
        self.exps_dir = exps_dir or at.exps_dir
        self.tuner_type = tuner_type or at.tuner_type
        self.trials = tuner_num_trials or at.tuner_num_trials
        self.early = at.tuner_early_stopping if tuner_early_stopping == -1 else tuner_early_stopping
        self.mbs = list(micro_batch_sizes) if micro_batch_sizes else None
        self.stages = list(stages if stages is not None else at.zero_stages)
        self.hbm = hbm_bytes
        self.metric = metric or at.metric
        self.fast = at.fast if fast is None else fast
        from .config import DEFAULT_TUNING_SPACE
        self.space = tuning_space if tuning_space is not None else DEFAULT_TUNING_SPACE
        self.records = []
        self.best = None

    # ---------------------------------------------------------------------------- memory model
    def feasible_stages(self):
        if not self.num_params:
            return self.stages
        return [s for s in self.stages if model_state_bytes(self.num_params, s, self.world) < 0.9 * self.hbm]

    def max_micro_batch(self, stage):
        """Largest micro-batch size the memory model admits (None: unknown -> the configured cap)."""
        at = self.at
        cap = at.max_train_micro_batch_size_per_gpu
        if at.max_train_batch_size:
            cap = min(cap, max(1, at.max_train_batch_size // max(1, self.world)))
        act = self.model_info.get("activation_mem_per_gpu")
        if not (self.num_params and act):
            return cap
        free = 0.9 * self.hbm - model_state_bytes(self.num_params, stage, self.world)
        return max(0, min(cap, int(free // act)))

    def micro_batch_candidates(self, stage):
        if self.mbs:
            hi = self.max_micro_batch(stage)
            return [m for m in self.mbs if m <= hi] if hi else list(self.mbs)
        lo, hi = self.at.min_train_micro_batch_size_per_gpu, self.max_micro_batch(stage)
        if hi < lo:
            return []
        n = max(1, self.at.num_tuning_micro_batch_sizes)
        if n == 1 or hi == lo:
            return [hi]
        vals = sorted({int(round(lo + (hi - lo) * i / (n - 1))) for i in range(n)})
        return vals

    # ----------------------------------------------------------------------------- experiments
    def experiments(self, stage=None, mbs_list=None):
        exps = []
        for st in ([stage] if stage is not None else self.feasible_stages()):
            for mb in (mbs_list if mbs_list is not None else self.micro_batch_candidates(st)):
                ov = {"zero_optimization": {"stage": st}, "train_micro_batch_size_per_gpu": mb}
                exps.append(Experiment(f"z{st}_mbs{mb}", ov))
        return exps

    def _space_experiments(self, stage, mbs):
        space = self.space.get(stage, {})
        if not space:
            return []
        keys = sorted(space)
        exps = []
        for vals in itertools.product(*(space[k] for k in keys)):
            ov = {"zero_optimization": {"stage": stage}, "train_micro_batch_size_per_gpu": mbs}
            for k, v in zip(keys, vals):
                _set_path(ov, k, v)
            tag = "_".join(f"{k.split('.')[-1].replace('stage3_', '')}{v}" for k, v in zip(keys, vals))
            exps.append(Experiment(f"z{stage}_mbs{mbs}_{tag}", ov))
        return exps

    def _config_for(self, exp):
        cfg = _deep_update(self.base, exp.overrides)
        cfg.pop("train_batch_size", None)
        if "gradient_accumulation_steps" not in exp.overrides and "train_batch_size" in self.base:
            cfg.pop("gradient_accumulation_steps", None)
        return cfg

    def _run_tuner(self, exps, run):
        if not exps:
            return None
        tuner = TUNERS[self.tuner_type](exps, run, metric=self.metric)
        return tuner.tune(self.trials, self.early)

    def model_info_profile_run(self, run_fn):
        """Profiling experiment (ZeRO-3, smallest micro-batch) whose engine reports model info."""
        if self.model_info.get("num_params") and self.model_info.get("activation_mem_per_gpu"):
            return self.model_info
        os.makedirs(self.results_dir, exist_ok=True)
        path = os.path.abspath(os.path.join(self.results_dir, "profile_model_info", "model_info.json"))
        os.makedirs(os.path.dirname(path), exist_ok=True)
        ov = {"zero_optimization": {"stage": 3}, "train_micro_batch_size_per_gpu": self.at.min_train_micro_batch_size_per_gpu,
              "autotuning": {"enabled": True, "model_info_path": path, "model_info": {"profile": True}}}
        try:
            run_fn(self._config_for(Experiment("profile_model_info", ov)))
        except Exception as e:  # noqa: BLE001 -- a profiling failure only disables the memory model
            self.records.append({"name": "profile_model_info", "error": repr(e)})
        if os.path.exists(path):
            with open(path) as f:
                self.model_info.update(json.load(f))
            self.num_params = self.model_info.get("num_params", self.num_params)
        return self.model_info

    def tune(self, run_fn, profile_model_info=False):
        """run_fn(config_dict) -> metric (higher is better) or raises (e.g. out of memory)."""
        def run(exp):
            t0 = time.time()
            try:
                m = run_fn(self._config_for(exp))
            except Exception as e:  # noqa: BLE001
                self.records.append({"name": exp.name, "config": exp.overrides, "metric": None, "error": repr(e),
                                     "secs": time.time() - t0})
                raise
            self.records.append({"name": exp.name, "config": exp.overrides, "metric": m, "secs": time.time() - t0})
            return m

        if profile_model_info:
            self.model_info_profile_run(run_fn)
        best = None
        for st in self.feasible_stages():
            b = self._run_tuner(self.experiments(st), run)
            if b is None:
                continue
            if not self.fast:
                mbs = b.overrides["train_micro_batch_size_per_gpu"]
                b2 = self._run_tuner(self._space_experiments(st, mbs), run)
                if b2 is not None and b2.metric > b.metric:
                    b = b2
            if best is None or b.metric > best.metric:
                best = b
            elif b.metric < 0.9 * best.metric:
                break  # higher stages only trade speed for memory from here on
        self.best = best
        self._write_results()
        return best

    def _write_results(self):
        os.makedirs(self.results_dir, exist_ok=True)
        best = self.best
        with open(os.path.join(self.results_dir, "summary.json"), "w") as f:
            json.dump({"metric": self.metric, "best": best.name if best else None,
                       "best_metric": best.metric if best else None,
                       "best_config": self.best_config(), "model_info": self.model_info,
                       "experiments": self.records}, f, indent=2)
        if best is not None:
            cfg = self.best_config()
            cfg.pop("autotuning", None)
            with open(os.path.join(self.results_dir, "ds_config_optimal.json"), "w") as f:
                json.dump(cfg, f, indent=2)

    def best_config(self):
        return self._config_for(self.best) if getattr(self, "best", None) else None

    def write_optimal_cmd(self, user_script, user_args=()):
        path = os.path.join(self.results_dir, "cmd_optimal.txt")
        cfg = os.path.abspath(os.path.join(self.results_dir, "ds_config_optimal.json"))
        with open(path, "w") as f:
            f.write(" ".join(["sxe", user_script] + list(user_args) + ["--deepspeed_config", cfg]) + "\n")
        return path


def scheduled_runner(user_script, user_args=(), exps_dir="autotuning_exps", nproc=1, timeout=1800,
                     start_step=3, end_step=5, metric="throughput", use_torchrun=True):
    """run_fn backed by scheduler.ResourceManager: each experiment is its own process group on
    ``nproc`` GPUs with logs / config / metrics under ``exps_dir/<name>/``."""
    from .scheduler import Experiment as SExp, ResourceManager
    rm = ResourceManager(user_script, user_args, num_gpus=nproc, exps_dir=exps_dir, metric=metric, exp_timeout=timeout,
                         start_profile_step=start_step, end_profile_step=end_step, use_torchrun=use_torchrun)
    count = [0]

    def run(cfg):
        count[0] += 1
        mb = cfg.get("train_micro_batch_size_per_gpu")
        st = cfg.get("zero_optimization", {}).get("stage")
        at = cfg.get("autotuning", {})
        if at.get("model_info_path"):
            # profiling run: the engine writes the model info; no metric is required
            e = SExp("profile_model_info", cfg, nproc)
            rm.schedule_experiments([e])
            rm.run()
            return 0.0
        return rm.run_one(SExp(f"exp{count[0]}_z{st}_mbs{mb}", cfg, nproc))
    run.manager = rm
    return run


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
