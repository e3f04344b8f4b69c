"""Data efficiency: per-sample difficulty analysis and curriculum-aware sampling.

Parity: reference runtime/data_pipeline/data_sampling/data_analyzer.py (``DataAnalyzer``: map a
metric over the dataset, save per-sample values + sorted index) and data_sampler.py
(``DeepSpeedDataSampler``: each global batch drawn from the samples whose difficulty is within the
current curriculum threshold, sharded over data-parallel ranks, deterministic per step).
"""
import os

import numpy as np
import torch


class DataAnalyzer:
    def __init__(self, dataset, metric_functions, metric_names, save_path, batch_size=1024):
        self.dataset, self.fns, self.names = dataset, list(metric_functions), list(metric_names)
        self.save_path = save_path
        self.batch_size = batch_size

    def run_map_reduce(self):
        os.makedirs(self.save_path, exist_ok=True)
        out = {}
        for fn, name in zip(self.fns, self.names):
            vals = np.array([float(fn(self.dataset[i])) for i in range(len(self.dataset))], dtype=np.float64)
            np.save(os.path.join(self.save_path, f"{name}_sample_to_metric.npy"), vals)
            np.save(os.path.join(self.save_path, f"{name}_index_sorted.npy"), np.argsort(vals, kind="stable"))
            out[name] = vals
        return out


class CurriculumDataSampler(torch.utils.data.Sampler):
    """Yields this rank's sample indices for each global batch; difficulty threshold from a
    ``CurriculumScheduler`` updated every batch."""

    def __init__(self, metric_values, scheduler, global_batch_size, dp_rank=0, dp_size=1, seed=1234,
                 total_steps=None):
        self.metric = np.asarray(metric_values)
        self.order = np.argsort(self.metric, kind="stable")
        self.sorted_vals = self.metric[self.order]
        self.sched = scheduler
        self.gbs = global_batch_size
        self.rank, self.size = dp_rank, dp_size
        self.seed = seed
        self.step = 0
        self.total_steps = total_steps

    def __len__(self):
        return (self.total_steps or (len(self.metric) // self.gbs)) * (self.gbs // self.size)

    def state_dict(self):
        return {"step": self.step, "curriculum": self.sched.get_state()}

    def load_state_dict(self, sd):
        self.step = sd["step"]
        self.sched.set_state(sd["curriculum"])

    def next_batch(self):
        self.step += 1
        thr = self.sched.update_difficulty(self.step)
        n_ok = int(np.searchsorted(self.sorted_vals, thr, side="right"))
        n_ok = max(n_ok, self.gbs)
        rng = np.random.default_rng(self.seed + self.step)
        picks = self.order[rng.choice(n_ok, size=self.gbs, replace=n_ok < self.gbs)]
        per = self.gbs // self.size
        return picks[self.rank * per:(self.rank + 1) * per].tolist()

    def __iter__(self):
        steps = self.total_steps or (len(self.metric) // self.gbs)
        for _ in range(steps):
            yield from self.next_batch()
