"""Data efficiency: per-sample difficulty analysis and curriculum-aware sampling.

Parity: reference runtime/data_pipeline/data_sampling/data_analyzer.py (``DataAnalyzer``: threaded
map over a worker's shard, file-based reduce into sample <-> metric indexes; ``DistributedDataAnalyzer``:
collective map-reduce with a distributed sample sort) and data_sampler.py
(``DeepSpeedDataSampler``: each global batch drawn from the samples whose difficulty is within the
current curriculum threshold, sharded over data-parallel ranks, deterministic per step).
"""
import os

import numpy as np
import torch


SINGLE, ACCUM = "single_value_per_sample", "accumulate_value_over_samples"


def _write_indexed(prefix, arrays, dtype):
    from .indexed_dataset import MMapIndexedDatasetBuilder, data_file_path, index_file_path
    b = MMapIndexedDatasetBuilder(data_file_path(prefix), dtype=dtype)
    for a in arrays:
        b.add_item(np.asarray(a))
        b.end_document()
    b.finalize(index_file_path(prefix))


def _metric_outputs(save_path, name, values, dtype, sample_dtype=np.int64):
    """Reduce outputs of one single-value metric (reference data_analyzer.py merge_map_results):
    ``{name}_sample_to_metric`` (value per sample), ``{name}_index_to_metric`` (distinct values,
    ascending), ``{name}_index_to_sample`` (samples per distinct value) and
    ``{name}_index_to_sample_percentile_merged`` (samples per percentile bucket) as Megatron mmap
    indexed datasets, plus .npy copies for direct numpy use."""
    d = os.path.join(save_path, name)
    os.makedirs(d, exist_ok=True)
    values = np.asarray(values)
    order = np.argsort(values, kind="stable")
    sorted_vals = values[order]
    distinct, starts = np.unique(sorted_vals, return_index=True)
    groups = np.split(order.astype(sample_dtype), starts[1:])
    _write_indexed(os.path.join(d, f"{name}_sample_to_metric"), [values.astype(dtype)], dtype)
    _write_indexed(os.path.join(d, f"{name}_index_to_metric"), [distinct.astype(dtype)], dtype)
    _write_indexed(os.path.join(d, f"{name}_index_to_sample"), groups, sample_dtype)
    pct = [order[int(len(order) * i / 100):int(len(order) * (i + 1) / 100)].astype(sample_dtype) for i in range(100)]
    _write_indexed(os.path.join(d, f"{name}_index_to_sample_percentile_merged"), pct, sample_dtype)
    np.save(os.path.join(save_path, f"{name}_sample_to_metric.npy"), values)
    np.save(os.path.join(save_path, f"{name}_index_sorted.npy"), order)
    return values


class DataAnalyzer:
    """Map a set of metrics over a dataset and reduce them into sample <-> metric indexes
    (reference data_sampling/data_analyzer.py ``DataAnalyzer``).

    Map: this worker (``worker_id`` of ``num_workers``, e.g. one per node) takes a contiguous shard
    of the dataset and splits it over ``num_threads`` threads; each writes its partial results under
    ``save_path/<metric>/worker<w>_thread<t>/``. ``single_value_per_sample`` metrics return one
    value per sample (from a batch: one value per batch row), ``accumulate_value_over_samples``
    metrics return an array summed over all samples (e.g. token frequencies).
    Reduce: the partial files of every worker/thread are merged (see ``_metric_outputs``).
    """

    def __init__(self, dataset, metric_functions, metric_names, save_path, batch_size=1024, num_workers=1,
                 worker_id=0, num_threads=1, metric_types=None, metric_dtypes=None, collate_fn=None):
        self.dataset, self.fns, self.names = dataset, list(metric_functions), list(metric_names)
        self.save_path = save_path
        self.batch_size = batch_size
        self.num_workers, self.worker_id, self.num_threads = num_workers, worker_id, num_threads
        self.types = list(metric_types or [SINGLE] * len(self.names))
        self.dtypes = list(metric_dtypes or [np.float64] * len(self.names))
        self.collate_fn = collate_fn

    def _shard(self, n, parts, i):
        per, rem = divmod(n, parts)
        lo = i * per + min(i, rem)
        return lo, lo + per + (1 if i < rem else 0)

    def _batch(self, idx):
        items = [self.dataset[j] for j in idx]
        return self.collate_fn(items) if self.collate_fn else items

    def _map_range(self, lo, hi):
        single = {n: [] for n, t in zip(self.names, self.types) if t == SINGLE}
        accum = {}
        for b0 in range(lo, hi, self.batch_size):
            idx = list(range(b0, min(hi, b0 + self.batch_size)))
            batch = self._batch(idx)
            for fn, name, typ in zip(self.fns, self.names, self.types):
                if typ == SINGLE:
                    v = fn(batch) if self.collate_fn else [fn(x) for x in batch]
                    single[name].append(np.asarray(v, dtype=np.float64).reshape(-1))
                else:
                    v = np.asarray(fn(batch) if self.collate_fn else sum(np.asarray(fn(x)) for x in batch))
                    accum[name] = accum[name] + v if name in accum else v
        return {n: (np.concatenate(v) if v else np.zeros(0)) for n, v in single.items()}, accum

    def run_map(self):
        import threading
        lo, hi = self._shard(len(self.dataset), self.num_workers, self.worker_id)
        results = [None] * self.num_threads

        def work(t):
            a, b = self._shard(hi - lo, self.num_threads, t)
            results[t] = self._map_range(lo + a, lo + b)
        ths = [threading.Thread(target=work, args=(t,)) for t in range(self.num_threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        for t, (single, accum) in enumerate(results):
            for name in self.names:
                d = os.path.join(self.save_path, name, f"worker{self.worker_id}_thread{t}")
                os.makedirs(d, exist_ok=True)
                if name in single:
                    np.save(os.path.join(d, "sample_to_metric.npy"), single[name])
                elif name in accum:
                    np.save(os.path.join(d, "metric_value.npy"), accum[name])

    def run_reduce(self):
        out = {}
        for name, typ, dt in zip(self.names, self.types, self.dtypes):
            parts = []
            for w in range(self.num_workers):
                for t in range(self.num_threads):
                    f = os.path.join(self.save_path, name, f"worker{w}_thread{t}",
                                     "sample_to_metric.npy" if typ == SINGLE else "metric_value.npy")
                    if os.path.exists(f):
                        parts.append(np.load(f))
            if typ == SINGLE:
                out[name] = _metric_outputs(self.save_path, name, np.concatenate(parts), dt)
            else:
                total = sum(parts)
                np.save(os.path.join(self.save_path, name, f"{name}_metric_value.npy"), total)
                out[name] = total
        return out

    def run_map_reduce(self, comm_group=None):
        self.run_map()
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            torch.distributed.barrier(group=comm_group)
            if torch.distributed.get_rank(comm_group) != 0:
                torch.distributed.barrier(group=comm_group)
                return None
            res = self.run_reduce()
            torch.distributed.barrier(group=comm_group)
            return res
        return self.run_reduce()


class DistributedDataAnalyzer:
    """Collective map-reduce (reference data_analyzer.py ``DistributedDataAnalyzer`` :455): every
    rank maps its shard in memory; the single-value metrics are globally sorted by a distributed
    sample sort (splitters from regular samples, one exchange of buckets, a local merge) and
    written rank by rank; accumulated metrics are all-reduced. No intermediate files."""

    def __init__(self, dataset, metric_functions, metric_names, save_path, batch_size=1024, metric_types=None,
                 metric_dtypes=None, collate_fn=None, comm_group=None):
        import torch.distributed as tdist
        self.g = comm_group
        self.rank, self.world = tdist.get_rank(comm_group), tdist.get_world_size(comm_group)
        self.inner = DataAnalyzer(dataset, metric_functions, metric_names, save_path, batch_size,
                                  num_workers=self.world, worker_id=self.rank, metric_types=metric_types,
                                  metric_dtypes=metric_dtypes, collate_fn=collate_fn)

    def _sample_sort(self, vals, ids):
        import torch.distributed as tdist
        order = np.lexsort((ids, vals))
        vals, ids = vals[order], ids[order]
        k = min(len(vals), 4 * self.world)
        local = vals[np.linspace(0, len(vals) - 1, k).astype(int)] if len(vals) else np.zeros(0)
        allsamp = [None] * self.world
        tdist.all_gather_object(allsamp, local, group=self.g)
        samp = np.sort(np.concatenate(allsamp))
        split = samp[np.linspace(0, len(samp) - 1, self.world + 1).astype(int)[1:-1]] if len(samp) else np.zeros(0)
        dest = np.searchsorted(split, vals, side="right")
        buckets = [(vals[dest == r], ids[dest == r]) for r in range(self.world)]
        allb = [None] * self.world
        tdist.all_gather_object(allb, buckets, group=self.g)
        v = np.concatenate([b[self.rank][0] for b in allb])
        i = np.concatenate([b[self.rank][1] for b in allb])
        o = np.lexsort((i, v))
        return v[o], i[o]

    def run_map_reduce(self):
        import torch.distributed as tdist
        a = self.inner
        lo, hi = a._shard(len(a.dataset), self.world, self.rank)
        single, accum = a._map_range(lo, hi)
        out = {}
        for name, typ, dt in zip(a.names, a.types, a.dtypes):
            if typ == SINGLE:
                vals = single[name]
                ids = np.arange(lo, hi, dtype=np.int64)
                sv, si = self._sample_sort(vals, ids)
                gathered = [None] * self.world
                tdist.all_gather_object(gathered, (vals, sv, si), group=self.g)
                if self.rank == 0:  # rank-ordered pieces: sample order and global metric order
                    full = np.concatenate([g[0] for g in gathered])
                    order = np.concatenate([g[2] for g in gathered])
                    assert np.array_equal(full[order], np.concatenate([g[1] for g in gathered]))
                    out[name] = _metric_outputs(a.save_path, name, full, dt)
            else:
                t = torch.as_tensor(accum.get(name, np.zeros(0)), dtype=torch.float64)
                tdist.all_reduce(t, group=self.g)
                if self.rank == 0:
                    d = os.path.join(a.save_path, name)
                    os.makedirs(d, exist_ok=True)
                    np.save(os.path.join(d, f"{name}_metric_value.npy"), t.numpy())
                    out[name] = t.numpy()
        tdist.barrier(group=self.g)
        return out if self.rank == 0 else None


class CurriculumDataSampler(torch.utils.data.Sampler):
    """Yields this rank's sample indices for each global batch; difficulty threshold from a
    ``CurriculumScheduler`` updated once per global batch = once per optimizer step (reference
    data_sampling/data_sampler.py:60,266: global_batch_size = micro x dp x gas). The global batch is
    laid out [gas, dp, micro]: this rank's indices come out as ``gas`` consecutive micro-batches."""

    def __init__(self, metric_values, scheduler, global_batch_size, dp_rank=0, dp_size=1, seed=1234,
                 total_steps=None, gradient_accumulation_steps=1, metric_name=None):
        self.metric_name = metric_name
        self.metric = np.asarray(metric_values)
        self.order = np.argsort(self.metric, kind="stable")
        self.sorted_vals = self.metric[self.order]
        self.sched = scheduler
        self.gbs = global_batch_size
        self.gas = max(1, int(gradient_accumulation_steps))
        self.rank, self.size = dp_rank, dp_size
        if self.gbs % (self.size * self.gas):
            raise ValueError(f"global batch {self.gbs} not divisible by dp {self.size} x gas {self.gas}")
        self.seed = seed
        self.step = 0
        self.total_steps = total_steps

    def __len__(self):
        return (self.total_steps or (len(self.metric) // self.gbs)) * (self.gbs // self.size)

    def state_dict(self):
        return {"step": self.step, "curriculum": self.sched.get_state()}

    def set_custom_curriculum_learning_schedule(self, schedule_func_dict):
        """{metric name: fn(global_step) -> difficulty} for metrics whose schedule_type is "custom"
        (reference data_sampling/data_sampler.py:117)."""
        fn = schedule_func_dict.get(self.metric_name) if self.metric_name is not None else None
        if fn is None and len(schedule_func_dict) == 1 and self.metric_name is None:
            fn = next(iter(schedule_func_dict.values()))
        if fn is not None:
            self.sched.set_custom_get_difficulty(fn)

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
        micro = self.gbs // (self.size * self.gas)
        return picks.reshape(self.gas, self.size, micro)[:, self.rank, :].reshape(-1).tolist()

    def __iter__(self):
        steps = self.total_steps or (len(self.metric) // self.gbs)
        for _ in range(steps):
            yield from self.next_batch()
