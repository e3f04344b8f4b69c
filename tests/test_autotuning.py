"""Autotuner: memory pruning of infeasible stages, grid / random / model-based search find the best
(synthetic) configuration, and a real in-process experiment measures engine throughput."""
import math
import pytest


def _synthetic(cfg):
    mbs = cfg["train_micro_batch_size_per_gpu"]
    st = cfg["zero_optimization"]["stage"]
    if mbs > 8:
        raise RuntimeError("OOM")
    return 100 * mbs - 10 * (mbs - 4) ** 2 + (5 if st == 2 else 0)


@pytest.mark.parametrize("tuner", ["gridsearch", "random", "model_based"])
def test_autotuner_finds_best(tuner, tmp_path):
    from shuffle_exchange_amd.autotuning import Autotuner
    at = Autotuner({"optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}, results_dir=str(tmp_path), tuner_type=tuner,
                   tuner_num_trials=40, tuner_early_stopping=None, micro_batch_sizes=[1, 2, 4, 8, 16], stages=(0, 1, 2, 3))
    best = at.tune(_synthetic)
    assert best.overrides["train_micro_batch_size_per_gpu"] == 8
    assert (tmp_path / "summary.json").exists()


def test_memory_pruning():
    from shuffle_exchange_amd.autotuning import Autotuner, model_state_bytes
    at = Autotuner({}, num_params=70e9, world_size=8)
    assert 0 not in at.feasible_stages() and 3 in at.feasible_stages()
    assert model_state_bytes(8e9, 3, 8) < model_state_bytes(8e9, 1, 8)


def test_engine_metric_probe(tmp_path):
    import json
    import torch
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    m = LlamaForCausalLM(llama_config("llama-tiny", num_hidden_layers=1))
    mp = tmp_path / "metric.json"
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
          "autotuning": {"enabled": True, "metric_path": str(mp), "start_profile_step": 1, "end_profile_step": 3,
                         "exit_after_profile": False}}
    eng, _, _, _ = sxe.initialize(model=m, config=ds)
    for _ in range(4):
        ids = torch.randint(0, 512, (2, 16))
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
    assert json.loads(mp.read_text())["throughput"] > 0


def test_autotuner_memory_model_and_tuning_space(tmp_path):
    """Model info drives the micro-batch candidates (activation bytes per sample vs free HBM), a
    stage whose model states do not fit is never run, and fast=False crosses the best micro-batch
    size with the stage's tuning space; the optimal config is written out."""
    import json
    from shuffle_exchange_amd.autotuning import Autotuner
    gib = 2 ** 30
    base = {"optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "train_batch_size": 64,
            "autotuning": {"fast": False, "num_tuning_micro_batch_sizes": 4, "max_train_micro_batch_size_per_gpu": 64,
                           "model_info": {"num_params": 40e9, "activation_mem_per_gpu": 4 * gib}}}
    seen = []

    def run(cfg):
        seen.append(cfg)
        zo = cfg["zero_optimization"]
        bonus = 3 if zo.get("stage3_defer_reduce") else 0
        return cfg["train_micro_batch_size_per_gpu"] + bonus

    at = Autotuner(base, world_size=8, results_dir=str(tmp_path), hbm_bytes=288 * gib, tuner_early_stopping=None)
    assert at.feasible_stages() == [2, 3]  # 40B params: ZeRO-0/1 model states exceed 0.9 x 288 GB per GPU
    free = 0.9 * 288 * gib - 40e9 * 18 / 8
    assert at.max_micro_batch(3) == int(free // (4 * gib))
    best = at.tune(run)
    assert {c["zero_optimization"]["stage"] for c in seen} == {2, 3}
    assert "train_batch_size" not in seen[0]
    assert best.overrides["zero_optimization"].get("stage3_defer_reduce") is True
    assert best.overrides["train_micro_batch_size_per_gpu"] == at.max_micro_batch(3)
    opt = json.loads((tmp_path / "ds_config_optimal.json").read_text())
    assert opt["zero_optimization"]["stage3_defer_reduce"] is True and "autotuning" not in opt


_USER_SCRIPT = '''
import argparse, json, torch
import shuffle_exchange_amd as sxe
from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
ap = argparse.ArgumentParser(); ap.add_argument("--deepspeed_config"); a = ap.parse_args()
cfg = json.load(open(a.deepspeed_config))
torch.manual_seed(0)
m = LlamaForCausalLM(llama_config("llama-tiny", num_hidden_layers=1))
eng, _, _, _ = sxe.initialize(model=m, config=cfg)
mb = eng.train_micro_batch_size_per_gpu()
for _ in range(20):
    ids = torch.randint(0, 512, (mb, 16))
    loss = eng(ids, labels=ids)
    eng.backward(loss)
    eng.step()
'''


def test_scheduler_runs_real_experiments(tmp_path, monkeypatch):
    """End to end on CPU: the profiling run writes model info from a real engine, then the
    ResourceManager runs experiments two at a time (one 'GPU' each), every one in its own directory
    with config, command, logs and the engine-written metrics."""
    import json
    from shuffle_exchange_amd.autotuning import Autotuner, scheduled_runner
    import os
    script = tmp_path / "train.py"
    script.write_text(_USER_SCRIPT)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.setenv("PYTHONPATH", root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    base = {"optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
            "autotuning": {"num_tuning_micro_batch_sizes": 2, "max_train_micro_batch_size_per_gpu": 4,
                           "zero_stages": [0, 1]}}
    run = scheduled_runner(str(script), exps_dir=str(tmp_path / "exps"), nproc=1, timeout=300, start_step=2,
                           end_step=4, use_torchrun=False)
    at = Autotuner(base, results_dir=str(tmp_path / "res"), tuner_early_stopping=None)
    best = at.tune(run, profile_model_info=True)
    info = at.model_info
    assert info["num_params"] > 0 and info["hidden_size"] > 0 and "activation_mem_per_gpu" in info
    assert best is not None and best.metric > 0
    names = sorted(p.name for p in (tmp_path / "exps").iterdir())
    assert "profile_model_info" in names and len(names) >= 5  # profile + 2 stages x 2 micro-batch sizes
    d = tmp_path / "exps" / names[0]
    for f in ("ds_config.json", "cmd.txt", "stdout.log", "stderr.log"):
        assert (d / f).exists()
    done = [e for e in run.manager.finished if e.metrics]
    assert all(e.metrics["throughput"] > 0 and e.metrics["latency"] > 0 for e in done)
    summary = json.loads((tmp_path / "res" / "summary.json").read_text())
    assert summary["best"] == best.name


def test_scheduler_parallel_slots(tmp_path):
    """Experiments needing one device each run side by side on a 2-device node; a 2-device one
    waits for both; a failing one is reported, not fatal."""
    from shuffle_exchange_amd.autotuning.scheduler import Experiment, ResourceManager
    script = tmp_path / "s.py"
    script.write_text("import json, os, sys, time\n"
                      "cfg = json.load(open(sys.argv[2]))\n"
                      "time.sleep(1.0)\n"
                      "if cfg.get('fail'): sys.exit(3)\n"
                      "json.dump({'throughput': float(cfg['v']), 'dev': os.environ['HIP_VISIBLE_DEVICES']},"
                      " open(cfg['autotuning']['metric_path'], 'w'))\n")
    import sys
    rm = ResourceManager(str(script), num_gpus=2, exps_dir=str(tmp_path / "e"), use_torchrun=True, poll_s=0.05)
    exps = [Experiment("a", {"v": 1}), Experiment("b", {"v": 5}), Experiment("c", {"v": 3}, num_gpus=2),
            Experiment("d", {"v": 9, "fail": True})]
    rm._command = lambda exp, cfg_path: [sys.executable, str(script), "--deepspeed_config", cfg_path]
    import time
    t0 = time.time()
    rm.schedule_experiments(exps)
    rm.run()
    assert time.time() - t0 < 3.9  # a||b, then c, then d would take >= 4 s serially
    assert rm.parse_results().name == "b"
    assert exps[2].metrics["dev"] == "0,1" and exps[3].error


def test_cost_model_tuner_finds_optimum_of_nonlinear_space():
    """Boosted-tree cost model (autotuning/cost_model.py, reference XGBoostCostModel) over generic
    flattened numeric knobs: on a 3-knob space with an interior optimum it reaches the best point
    well before exhausting the space, for throughput (max) and latency (min) metrics."""
    import itertools
    from shuffle_exchange_amd.autotuning.autotuner import Experiment, ModelBasedTuner
    from shuffle_exchange_amd.autotuning.cost_model import ConfigFeaturizer, flatten
    space = [{"train_micro_batch_size_per_gpu": m, "zero_optimization": {"stage": s, "reduce_bucket_size": b}}
             for m, s, b in itertools.product([1, 2, 4, 8, 16, 32], [0, 1, 2, 3], [1e7, 5e7, 2e8])]

    def tput(e):
        o = e.overrides
        m, s, b = o["train_micro_batch_size_per_gpu"], o["zero_optimization"]["stage"], o["zero_optimization"]["reduce_bucket_size"]
        return 100 - (math.log2(m) - 3) ** 2 * 6 - abs(s - 2) * 9 - abs(math.log10(b) - 7.7) * 4

    exps = [Experiment(f"e{i}", c) for i, c in enumerate(space)]
    f = ConfigFeaturizer([e.overrides for e in exps])
    assert f.keys == sorted(flatten(space[0]))
    best = max(exps, key=tput)
    hits = 0
    for seed in range(5):
        for e in exps:
            e.metric = None
        t = ModelBasedTuner(exps, tput, metric="throughput", seed=seed, warmup=4)
        t.tune(n_trials=30)
        hits += t.best is best
    assert hits >= 4
    for e in exps:
        e.metric = None
    t = ModelBasedTuner(exps, lambda e: 1.0 / tput(e), metric="latency", seed=0, warmup=4)
    assert t.tune(n_trials=30) is best
