"""data_efficiency engine wiring (reference runtime/engine.py:384-388, 698-741, 1954-1962, 2064-2065):
curriculum data sampling from a per-sample difficulty metric and random layerwise token drop."""
import os

import numpy as np
import torch

from .dist_utils import run_dist


def _case_rltd(rank, world):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.runtime.data_pipeline import RandomLayerTokenDrop
    from ._dist_cases import tiny_llama
    model, cfg = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
          "zero_optimization": {"stage": 2},
          "data_efficiency": {"enabled": True, "seed": 3, "data_routing": {"enabled": True, "random_ltd": {
              "enabled": True, "random_ltd_layer_num": 1, "random_ltd_layer_id": [1],
              "random_ltd_schedule": {"min_value": 8, "max_value": 32, "schedule_type": "fixed_linear",
                                      "schedule_config": {"require_steps": 2, "seq_per_step": 8}}}}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    wrapped = [m for m in eng.module.modules() if isinstance(m, RandomLayerTokenDrop)]
    seen = []
    wrapped[0].layer.register_forward_pre_hook(lambda m, a: seen.append(a[0].shape[1]))
    losses = []
    g = torch.Generator().manual_seed(5)
    for _ in range(5):
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    eng.eval()
    with torch.no_grad():
        eng(ids, labels=ids)
    return {"n_wrapped": len(wrapped), "seen": seen, "losses": losses}


def test_random_ltd_engine_wiring():
    for r in run_dist(_case_rltd, 2):
        assert r["n_wrapped"] == 1
        # kept tokens follow the schedule (8 -> 16 -> 24 tokens), then the full sequence in eval
        assert r["seen"][:5] == [8, 8, 16, 16, 24] and r["seen"][-1] == 32, r["seen"]
        assert all(x == x for x in r["losses"])


class _DS(torch.utils.data.Dataset):
    def __len__(self):
        return 64

    def __getitem__(self, i):
        return torch.full((8,), i, dtype=torch.long)


def _case_curriculum(rank, world, metric_path):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import tiny_llama
    model, _ = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "SGD", "params": {"lr": 1e-3}},
          "data_efficiency": {"enabled": True, "seed": 7, "data_sampling": {"enabled": True, "curriculum_learning": {
              "enabled": True, "curriculum_metrics": {"seqlen": {
                  "index_to_metric_path": metric_path, "difficulty_type": "value", "clustering_type": "single_cluster",
                  "min_difficulty": 10, "max_difficulty": 63, "schedule_type": "fixed_linear",
                  "schedule_config": {"total_curriculum_step": 8, "difficulty_step": 1}}}}}}}
    eng, _, loader, _ = sxe.initialize(model=model, config=ds, training_data=_DS())
    out = []
    it = iter(loader)
    for _ in range(6):
        b = next(it)
        out.append(b[:, 0].tolist())
    return {"batches": out}


def test_curriculum_sampler_engine_wiring(tmp_path):
    metric = np.arange(64, dtype=np.float64)  # difficulty == sample index
    path = str(tmp_path / "seqlen_sample_to_metric.npy")
    np.save(path, metric)
    res = run_dist(_case_curriculum, 2, path)
    # every rank draws its half of each global batch from samples within the current difficulty
    for step in range(6):
        both = res[0]["batches"][step] + res[1]["batches"][step]
        thr = max(10 + int((step + 1) / 8 * 53), 4)
        assert max(both) <= max(thr, 3), (step, both, thr)
    assert max(res[0]["batches"][0] + res[1]["batches"][0]) <= 16


def test_curriculum_difficulty_advances_per_optimizer_step():
    """gas > 1: the difficulty schedule advances once per GLOBAL batch (micro x dp x gas), and the
    rank's share of one global batch comes out as gas micro-batches (reference data_sampler.py:60,266;
    ADVICE r02). Before the fix it advanced once per micro-batch, gas times too fast."""
    from shuffle_exchange_amd.runtime.data_pipeline import CurriculumDataSampler, CurriculumScheduler
    metric = np.arange(256, dtype=np.float64)
    cfg = {"curriculum_type": "seqlen", "min_difficulty": 16, "max_difficulty": 255, "schedule_type": "fixed_linear",
           "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 1}}
    micro, dp, gas = 2, 2, 4
    samplers = [CurriculumDataSampler(metric, CurriculumScheduler(dict(cfg)), micro * dp * gas, dp_rank=r, dp_size=dp,
                                      gradient_accumulation_steps=gas, total_steps=6) for r in range(dp)]
    streams = [list(iter(s)) for s in samplers]
    per_step = micro * gas
    for step in range(6):
        thr = CurriculumScheduler(dict(cfg)).update_difficulty(step + 1)
        both = sum((st[step * per_step:(step + 1) * per_step] for st in streams), [])
        assert len(set(both)) == len(both) == micro * dp * gas  # one global batch, no overlap
        assert max(both) <= max(thr, micro * dp * gas - 1), (step, max(both), thr)
    assert samplers[0].step == 6  # one scheduler step per optimizer step, not per micro-batch


class _Toks(torch.utils.data.Dataset):
    def __init__(self, n=97):
        g = torch.Generator().manual_seed(0)
        self.items = [torch.randint(0, 16, (int(torch.randint(2, 20, (1,), generator=g)),), generator=g)
                      for _ in range(n)]

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def _seqlen(x):
    return len(x)


def _vocab(x):
    return np.bincount(x.numpy(), minlength=16)


def _check_outputs(path, ds):
    from shuffle_exchange_amd.runtime.data_pipeline.indexed_dataset import MMapIndexedDataset
    lens = np.array([len(x) for x in ds.items])
    s2m = MMapIndexedDataset(os.path.join(path, "seqlen", "seqlen_sample_to_metric"))[0]
    assert np.array_equal(s2m, lens)
    i2m = MMapIndexedDataset(os.path.join(path, "seqlen", "seqlen_index_to_metric"))[0]
    assert np.array_equal(i2m, np.unique(lens))
    i2s = MMapIndexedDataset(os.path.join(path, "seqlen", "seqlen_index_to_sample"))
    for k, v in enumerate(i2m):
        assert np.array_equal(np.sort(i2s[k]), np.nonzero(lens == v)[0])
    pct = MMapIndexedDataset(os.path.join(path, "seqlen", "seqlen_index_to_sample_percentile_merged"))
    assert sum(len(pct[k]) for k in range(len(pct))) == len(lens)
    vocab = np.load(os.path.join(path, "vocab", "vocab_metric_value.npy"))
    assert np.array_equal(vocab, np.bincount(torch.cat(ds.items).numpy(), minlength=16))


def test_data_analyzer_map_reduce(tmp_path):
    """Threaded map over 3 workers' shards + file reduce == brute force; outputs are indexed datasets."""
    from shuffle_exchange_amd.runtime.data_pipeline import DataAnalyzer
    ds = _Toks()
    kw = dict(metric_functions=[_seqlen, _vocab], metric_names=["seqlen", "vocab"], save_path=str(tmp_path),
              batch_size=8, num_workers=3, num_threads=2,
              metric_types=["single_value_per_sample", "accumulate_value_over_samples"],
              metric_dtypes=[np.int64, np.int64])
    for w in range(3):
        DataAnalyzer(ds, worker_id=w, **kw).run_map()
    DataAnalyzer(ds, worker_id=0, **kw).run_reduce()
    _check_outputs(str(tmp_path), ds)


def _case_dist_analyzer(rank, world, path):
    from shuffle_exchange_amd.runtime.data_pipeline import DistributedDataAnalyzer
    ds = _Toks()
    DistributedDataAnalyzer(ds, [_seqlen, _vocab], ["seqlen", "vocab"], path, batch_size=5,
                            metric_types=["single_value_per_sample", "accumulate_value_over_samples"],
                            metric_dtypes=[np.int64, np.int64]).run_map_reduce()
    return True


def test_distributed_data_analyzer(tmp_path):
    """Collective map-reduce over 3 gloo ranks (distributed sample sort) == brute force."""
    from .dist_utils import run_dist
    run_dist(_case_dist_analyzer, 3, str(tmp_path))
    _check_outputs(str(tmp_path), _Toks())


def _case_rltd_ac(rank, world, ac):
    """Parameters after one random-LTD accumulation window (2 micro-steps, SGD) with or without full
    activation checkpointing: equal gradients give equal parameters."""
    import shuffle_exchange_amd as sxe
    from ._dist_cases import tiny_llama
    model, cfg = tiny_llama(0, activation_checkpointing=ac, ac_policy="full")
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2,
          "optimizer": {"type": "SGD", "params": {"lr": 0.5}}, "zero_optimization": {"stage": 0},
          "data_efficiency": {"enabled": True, "seed": 3, "data_routing": {"enabled": True, "random_ltd": {
              "enabled": True, "random_ltd_layer_num": 2, "random_ltd_layer_id": [0, 1],
              "random_ltd_schedule": {"min_value": 8, "max_value": 32, "schedule_type": "fixed_linear",
                                      "schedule_config": {"require_steps": 100, "seq_per_step": 8}}}}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(5)
    for _ in range(2):  # one accumulation window of two micro-steps
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        eng.backward(eng(ids, labels=ids))
        eng.step()
    return {"params": {n: p.detach().clone() for n, p in eng.module.named_parameters()},
            "consumed": eng.random_ltd_scheduler.consumed_layer_tokens}


def test_random_ltd_with_full_activation_checkpointing_matches():
    """The recompute of a checkpointed random-LTD layer keeps the forward's tokens (draws keyed by
    step / micro-step / layer, not a counter), so training equals the uncheckpointed run and the
    consumed-token count is not doubled."""
    a = run_dist(_case_rltd_ac, 1, False)[0]
    b = run_dist(_case_rltd_ac, 1, True)[0]
    assert a["consumed"] == b["consumed"] == 2 * 2 * 2 * 8
    moved = 0
    for n in a["params"]:
        assert torch.allclose(a["params"][n], b["params"][n], atol=1e-6, rtol=1e-5), n
        moved += int(not torch.equal(a["params"][n], tiny_llama_param(n)))
    assert moved > 0


def tiny_llama_param(name):
    from ._dist_cases import tiny_llama
    return dict(tiny_llama(0)[0].named_parameters())[name.replace(".layer.", ".")].detach()
