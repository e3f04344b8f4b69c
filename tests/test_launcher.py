"""Launcher: hostfile parsing, include/exclude resource filters, world-info round trip, multi-node
command construction, and a real 2-rank local launch (gloo) through runner -> launch -> script."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hostfile_and_filters():
    from shuffle_exchange_amd.launcher.runner import parse_hostfile, parse_resource_filter
    pool = parse_hostfile(["# cluster", "worker-0 slots=8", "worker-1 slots=8  # second", ""])
    assert dict(pool) == {"worker-0": 8, "worker-1": 8}
    inc = parse_resource_filter(pool, include_str="worker-0:0,1@worker-1")
    assert inc == {"worker-0": [0, 1], "worker-1": list(range(8))}
    exc = parse_resource_filter(pool, exclude_str="worker-1:0,7")
    assert exc["worker-1"] == [1, 2, 3, 4, 5, 6] and exc["worker-0"] == list(range(8))
    assert "worker-1" not in parse_resource_filter(pool, exclude_str="worker-1")
    with pytest.raises(ValueError):
        parse_resource_filter(pool, include_str="nope")
    with pytest.raises(ValueError):
        parse_hostfile(["a slots=1", "a slots=2"])


def test_world_info_and_multinode_cmds(tmp_path):
    from shuffle_exchange_amd.launcher import runner
    wi = {"a": [0, 1], "b": [0, 1]}
    assert runner.decode_world_info(runner.encode_world_info(wi)) == wi
    hf = tmp_path / "hostfile"
    hf.write_text("a slots=2\nb slots=2\n")
    args = runner.parse_args(["-H", str(hf), "--launcher", "ssh", "train.py", "--x", "1"])
    cmds = runner.multinode_commands(args, wi, "a")
    assert len(cmds) == 2 and cmds[0][:2] == ["ssh", "a"] and "--node_rank=1" in cmds[1][2]
    assert "train.py --x 1" in cmds[0][2]


SCRIPT = """
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
with open(os.path.join(sys.argv[-1], f"r{dist.get_rank()}.txt"), "w") as f:
    f.write(f"{os.environ['LOCAL_RANK']} {os.environ['WORLD_SIZE']} {t.item()}")
dist.destroy_process_group()
"""


def test_local_launch_two_ranks(tmp_path):
    script = tmp_path / "s.py"
    script.write_text(SCRIPT)
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "shuffle_exchange_amd.launcher.runner", "-H", "/nonexistent",
                        "--num_gpus", "2", "--master_port", "29677", "--no_local_rank", str(script), str(tmp_path)],
                       env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    outs = sorted((tmp_path / f"r{i}.txt").read_text() for i in range(2))
    assert outs == ["0 2 3.0", "1 2 3.0"]


def test_env_report_runs():
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bin", "sxe_report")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "torch version" in r.stdout and "cpu (Adam" in r.stdout


TRAIN_SCRIPT = """
import os, sys, time
sys.path.insert(0, os.environ["SXE_ROOT"])
import torch
import shuffle_exchange_amd as sxe
from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
sxe.init_distributed(dist_backend="gloo", verbose=False)
cfg = llama_config("llama-tiny")
model = LlamaForCausalLM(cfg)
eng, _, _, _ = sxe.initialize(model=model, config={"train_micro_batch_size_per_gpu": 1,
    "zero_optimization": {"stage": 1}, "optimizer": {"type": "SGD", "params": {"lr": 0.1}}})
ids = torch.randint(0, cfg.vocab_size, (1, 16))
for step in range(6):
    loss = eng(ids, labels=ids)
    eng.backward(loss)
    eng.step()
open(os.path.join(sys.argv[-1], f"done{eng.global_rank}"), "w").close()
"""


def test_fault_injection_kill_triggers_launcher_fail_fast(tmp_path):
    """SXE_FAULT=kill@1:2: rank 1 dies at step 2; the launcher tears the job down with its status
    instead of leaving rank 0 blocked in the next collective (reference launch.py:338-359)."""
    script = tmp_path / "t.py"
    script.write_text(TRAIN_SCRIPT)
    env = dict(os.environ, PYTHONPATH=ROOT, SXE_ROOT=ROOT, SXE_FAULT="kill@1:2")
    r = subprocess.run([sys.executable, "-m", "shuffle_exchange_amd.launcher.runner", "-H", "/nonexistent",
                        "--num_gpus", "2", "--master_port", "29679", "--no_local_rank", str(script), str(tmp_path)],
                       env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 17, r.stdout[-3000:]
    assert "[sxe fault] kill on rank 1 at step 2" in r.stdout
    assert not (tmp_path / "done0").exists() and not (tmp_path / "done1").exists()


def test_fault_rules_parse():
    from shuffle_exchange_amd.utils import fault
    os.environ["SXE_FAULT"] = "raise@*:4; kill@3:9"
    try:
        assert fault._rules() == [("raise", "*", 4), ("kill", "3", 9)]
        import pytest
        with pytest.raises(fault.InjectedFault):
            fault.maybe_inject(0, 4)
        fault.maybe_inject(0, 5)
    finally:
        del os.environ["SXE_FAULT"]


FLAKY_SCRIPT = """
import os, sys
sys.path.insert(0, os.environ["SXE_ROOT"])
import torch, torch.distributed as dist
dist.init_process_group("gloo")
attempt = int(os.environ["SXE_RESTART_COUNT"])
if attempt == 0 and dist.get_rank() == 1:
    os._exit(3)  # first incarnation: rank 1 crashes
t = torch.ones(1)
dist.all_reduce(t)
open(os.path.join(sys.argv[-1], f"ok{dist.get_rank()}_{attempt}"), "w").write(str(t.item()))
dist.destroy_process_group()
"""


def test_launcher_restarts_failed_worker_group(tmp_path):
    """--max_restarts (elastic agent policy): the failed group is torn down and restarted; the
    second incarnation (SXE_RESTART_COUNT=1) completes."""
    script = tmp_path / "f.py"
    script.write_text(FLAKY_SCRIPT)
    env = dict(os.environ, PYTHONPATH=ROOT, SXE_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-m", "shuffle_exchange_amd.launcher.runner", "-H", "/nonexistent",
                        "--num_gpus", "2", "--master_port", "29683", "--no_local_rank", "--max_restarts", "2",
                        str(script), str(tmp_path)],
                       env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    assert (tmp_path / "ok0_1").read_text() == "2.0" and (tmp_path / "ok1_1").exists()
    assert "restart 1/2" in r.stdout


def test_elastic_agent_importable():
    from shuffle_exchange_amd.elasticity.elastic_agent import SXEElasticAgent
    assert SXEElasticAgent.__name__ == "SXEElasticAgent"
