"""bench.py driver contract, rehearsed on the CPU: two ranks under torch.distributed.run (gloo),
tiny Llama, one JSON line from rank 0 with the required keys and whole-job token accounting."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_cpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29631", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--model", "llama-tiny", "--device", "cpu", "--seq", "64", "--mbs", "2", "--gas", "2"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 2 * 2 * 2 and out["config"]["seq_len"] == 64
    tokens = 2 * 2 * 2 * 64 * 2
    assert abs(out["value"] - tokens / (out["ms_per_step"] * 2 / 1000.0)) / out["value"] < 0.01
    assert out["valid_for_metric"] is False  # tiny model on CPU is never a metric number


import pytest  # noqa: E402


@pytest.mark.parametrize("config,model,extra", [
    ("llama8b-z3-default", "llama-tiny", []),
    ("mixtral-ep", "mixtral-tiny", []),
    ("llama70b-infinity", "llama-tiny", ["--layers", "2"]),
    ("llama8b-sp32k", "llama-tiny", ["--seq", "128"]),
])
def test_bench_configs_two_ranks_cpu(tmp_path, config, model, extra):
    """Every BASELINE config's harness under torch.distributed.run with 2 gloo ranks: one JSON line,
    the config's parallelism (ep2 / sp2 / offload), its ZeRO knobs, the measured comm volume next to
    the analytic model."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    port = {"llama8b-z3-default": 29641, "mixtral-ep": 29643, "llama70b-infinity": 29645, "llama8b-sp32k": 29647}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port[config]), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--config", config, "--model", model, "--device", "cpu",
           "--mbs", "1", "--gas", "2"] + extra
    if "--seq" not in extra:
        cmd += ["--seq", "64"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    out = json.loads(lines[0])
    cfg = out["config"]
    assert cfg["name"] == config and out["n_gpus"] == 2 and out["valid_for_metric"] is False
    assert "zero_optimization" in cfg and cfg["zero_optimization"]["stage"] in (2, 3)
    meas, model_ = out["comm_measured"], out["comm_model"]
    if config == "mixtral-ep":
        assert cfg["expert_parallel_size"] == 2 and "ep2" in cfg["parallelism"]
        assert meas["all_to_all_single"]["calls_per_step"] > 0
    if config == "llama8b-sp32k":
        assert cfg["sequence_parallel_size"] == 2 and out["scaling"] == "strong"
        assert cfg["global_batch"] == 2  # one sequence per SP group per micro-step x gas 2
        assert meas["all_to_all_single"]["calls_per_step"] > 0
    if config == "llama70b-infinity":
        assert cfg["zero_optimization"]["offload_optimizer"]["device"] == "cpu"
    if config == "llama8b-z3-default":
        assert cfg["zero_knobs"] == "reference"
        # 2 gathers (fwd + bwd) and 1 reduce-scatter per micro-step: the analytic model agrees with the
        # bytes the facade counted
        for op in ("all_gather_into_tensor", "reduce_scatter_tensor"):
            assert meas[op]["bytes_per_step"] == model_[op], (op, meas[op], model_[op])


def test_bench_tuned_zero3_comm_model_matches_measured(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29649", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--model", "llama-tiny", "--device", "cpu", "--seq", "64", "--mbs", "1", "--gas", "2"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    meas, model_ = out["comm_measured"], out["comm_model"]
    assert out["config"]["zero_knobs"] == "tuned"
    # tuned: ONE gather of the model per step and ONE deferred reduce-scatter per step
    for op in ("all_gather_into_tensor", "reduce_scatter_tensor"):
        assert meas[op]["bytes_per_step"] == model_[op], (op, meas[op], model_[op])


CONFIGS = ["llama8b-z3", "llama8b-z3-default", "mixtral-ep", "llama70b-infinity", "llama8b-sp32k"]


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("config", CONFIGS)
def test_bench_configs_wide_cpu(tmp_path, config, world):
    """Every BASELINE config at the driver's W=4 and W=8 over gloo, with models whose head/expert
    counts make SP=8 / EP=8 legal (llama-tiny8: 16 q / 8 kv heads, mixtral-tiny8: 8 experts): one
    JSON line, the config's parallelism degree equal to W where it scales with W, the measured
    ZeRO collective bytes equal to the analytic model, and the first step's collective fingerprint
    identical on every rank (bench.py raises otherwise)."""
    model = "mixtral-tiny8" if config == "mixtral-ep" else "llama-tiny8"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    port = 29700 + 2 * CONFIGS.index(config) + (0 if world == 4 else 20)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus",
           str(world), "--steps", "2", "--warmup", "1", "--config", config, "--model", model, "--device", "cpu",
           "--mbs", "1", "--gas", "2", "--seq", "128"]
    if config == "llama70b-infinity":
        cmd += ["--layers", "2"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    out = json.loads(lines[0])
    cfg = out["config"]
    assert out["n_gpus"] == world and cfg["name"] == config and out["valid_for_metric"] is False
    diag = out["diagnostics"]
    assert diag["fingerprint_first_step"]["ranks_agree"] and diag["fingerprint_first_step"]["collectives"] > 0
    assert diag["communicators"] >= 1
    if config == "mixtral-ep":
        assert cfg["expert_parallel_size"] == world and f"ep{world}" in cfg["parallelism"]
    elif config == "llama8b-sp32k":
        assert cfg["sequence_parallel_size"] == world and cfg["global_batch"] == 2
    else:
        assert f"dp{world}" in cfg["parallelism"] and cfg["global_batch"] == world * 2
    meas, model_ = out["comm_measured"], out["comm_model"]
    assert model_, out
    for op, b in model_.items():
        assert meas[op]["bytes_per_step"] == b, (op, meas[op], b)


def test_auto_ac_policy_partial_mlp_layers():
    """288 GB: Llama-3-8B at 32k tokens on one GPU checkpoints the MLP of only part of the layers;
    from 2 GPUs (16k tokens each) nothing is recomputed."""
    import bench
    pol, n = bench.auto_ac_policy("llama3-8b", None, 32768, 1, 3)
    assert pol == "mlp" and 0 < n < 32
    assert bench.auto_ac_policy("llama3-8b", None, 16384, 2, 3) == ("none", None)
    assert bench.auto_ac_policy("llama3-8b", None, 16384, 1, 3)[0] == "none"


def test_llama_ac_layers_covers_first_layers():
    import torch
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    cfg = llama_config("llama-tiny", num_hidden_layers=4, activation_checkpointing=True, ac_policy="mlp", ac_layers=3)
    m = LlamaForCausalLM(cfg)
    assert [layer.ckpt_mlp for layer in m.layers] == [True, True, True, False]
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    m(ids, labels=ids).backward()
    assert all(p.grad is not None for p in m.parameters() if p.requires_grad)
