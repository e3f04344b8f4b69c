"""Engine observability and config honesty: the throughput timer is driven (samples/s, tokens/s,
TFLOP/s), the monitor receives train loss / lr / loss scale / throughput / timer events (reference
runtime/engine.py:2068, 2204, 2451-2575), and accepted-but-ignored config knobs warn."""
import csv
import os

import torch

from .dist_utils import run_dist


def _case_monitor(rank, world, out_dir):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny")
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "steps_per_print": 2,
          "wall_clock_breakdown": True,
          "zero_optimization": {"stage": 2}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
          "csv_monitor": {"enabled": True, "output_path": out_dir, "job_name": "job"}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    eng.tput_timer.start_step = 1
    ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=torch.Generator().manual_seed(rank))
    for _ in range(4 * 2):
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
    t = eng.tput_timer
    return {"seq": t.seq_len, "sps": t.avg_samples_per_sec(), "tps": t.avg_tokens_per_sec(), "tfl": t.avg_tflops(),
            "steps": t.global_step_count, "report": t.last_report}


def test_throughput_timer_and_monitor_events(tmp_path):
    res = run_dist(_case_monitor, 2, str(tmp_path))
    r = res[0]
    assert r["steps"] == 4 and r["seq"] == 32
    assert r["sps"] > 0 and abs(r["tps"] - 32 * r["sps"]) < 1e-6 * r["tps"] and r["tfl"] > 0
    assert r["report"] and r["report"]["tokens_per_sec"] > 0
    d = os.path.join(tmp_path, "job")
    files = set(os.listdir(d))
    for name in ("train_loss", "lr", "loss_scale", "tokens_per_sec", "samples_per_sec", "tflops_per_gpu",
                 "elapsed_time_ms_forward", "elapsed_time_ms_backward", "elapsed_time_ms_step"):
        assert f"Train_Samples_{name}.csv" in files, (name, files)
    with open(os.path.join(d, "Train_Samples_train_loss.csv")) as f:
        rows = list(csv.reader(f))
    assert len(rows) == 1 + 4  # header + one row per optimizer step
    losses = [float(x[1]) for x in rows[1:]]
    assert all(l == l and l > 0 for l in losses)
    with open(os.path.join(d, "Train_Samples_tokens_per_sec.csv")) as f:
        assert len(list(csv.reader(f))) == 1 + 2  # reported every steps_per_print=2 steps


def test_ignored_knobs_warn(caplog):
    from shuffle_exchange_amd.runtime.config import SXEConfig
    cfg = SXEConfig({"train_micro_batch_size_per_gpu": 1, "sparse_gradients": True,
                     "zero_optimization": {"stage": 3, "sub_group_size": 1000, "round_robin_gradients": True}})
    keys = [k for k, _ in cfg.ignored_knobs]
    assert "zero_optimization.sub_group_size" in keys
    assert "zero_optimization.round_robin_gradients" in keys
    assert "sparse_gradients" in keys
    quiet = SXEConfig({"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": 3}})
    assert quiet.ignored_knobs == []
