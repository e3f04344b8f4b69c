"""Per-rank host resources of the offload tier (utils/host_resources.py): thread-team sizing under
torchrun's OMP_NUM_THREADS=1, CPU shares per rank / NUMA node, and the host-memory pre-flight."""
import json
import os
import subprocess
import sys

import pytest

from shuffle_exchange_amd.utils import host_resources as hr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_share_split_when_unbound():
    cpus = list(range(64))
    shares = [hr.rank_cpu_share(r, 8, mask=cpus, online=cpus)[0] for r in range(8)]
    assert all(len(s) == 8 for s in shares)
    assert len(set(c for s in shares for c in s)) == 64  # disjoint, covering the host


def test_share_keeps_launcher_binding():
    share, how = hr.rank_cpu_share(3, 8, mask=[8, 9, 10], online=range(64))
    assert share == [8, 9, 10] and how == "inherited"


def test_share_numa_node_slices():
    online = list(range(128))
    node1 = list(range(64, 128))
    s0, how = hr.rank_cpu_share(4, 8, mask=online, online=online, numa=node1, ranks_on_node=[4, 5, 6, 7])
    s3, _ = hr.rank_cpu_share(7, 8, mask=online, online=online, numa=node1, ranks_on_node=[4, 5, 6, 7])
    assert how == "numa" and s0 == list(range(64, 80)) and s3 == list(range(112, 128))


def test_threads_ignore_torchrun_placeholder():
    share = list(range(24))
    assert hr.host_threads(share, omp_env="1", local_world=8, explicit="") == 24   # torchrun's default
    assert hr.host_threads(share, omp_env="1", local_world=1, explicit="") == 1    # a deliberate 1
    assert hr.host_threads(share, omp_env="16", local_world=8, explicit="") == 16  # a budget caps
    assert hr.host_threads(share, omp_env=None, local_world=8, explicit="") == 24
    assert hr.host_threads(share, omp_env="1", local_world=8, explicit="5") == 5


def test_preflight_message_names_the_need():
    with pytest.raises(MemoryError) as e:
        hr.preflight_host_memory(140 * 2**30, "ZeRO-Offload optimizer tier (cpu)", local_world=8,
                                 available=512 * 2**30)
    msg = str(e.value)
    assert "140.0 GiB" in msg and "x 8 local ranks = 1120.0 GiB" in msg and "512.0 GiB available" in msg
    assert "offload_optimizer.ratio" in msg
    hr.preflight_host_memory(10 * 2**30, "x", local_world=8, available=512 * 2**30)  # fits: no raise


def test_torchrun_eight_ranks_each_get_their_share(tmp_path):
    """Under torchrun --nproc-per-node 8 (which exports OMP_NUM_THREADS=1), every rank's host-Adam
    team is at least cores/8 and the ranks' CPU sets are disjoint."""
    script = tmp_path / "probe.py"
    script.write_text(
        "import json, os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from shuffle_exchange_amd.ops import native\n"
        "native.require_cpu()\n"
        "import torch\n"
        "from shuffle_exchange_amd.utils.host_resources import configure_host_threads\n"
        "n = configure_host_threads()\n"
        "print('PROBE ' + json.dumps({'rank': int(os.environ['RANK']), 'threads': n,\n"
        "      'omp': int(torch.ops.sxe_cpu.num_threads()), 'cpus': sorted(os.sched_getaffinity(0)),\n"
        "      'env_omp': os.environ.get('OMP_NUM_THREADS')}), flush=True)\n")
    env = {k: v for k, v in os.environ.items() if k not in ("OMP_NUM_THREADS", "SXE_HOST_ADAM_THREADS")}
    env["PYTHONPATH"] = ROOT
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", "29671", str(script)]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    probes = [json.loads(l.split("PROBE ", 1)[1]) for l in r.stdout.splitlines() if "PROBE " in l]
    assert len(probes) == 8
    cores = len(os.sched_getaffinity(0))
    for p in probes:
        assert p["env_omp"] == "1"  # torchrun's placeholder was there ...
        assert p["threads"] >= max(1, cores // 8) and p["omp"] == p["threads"]  # ... and not obeyed
    if cores >= 8:
        sets = [set(p["cpus"]) for p in probes]
        assert sum(len(s) for s in sets) == len(set().union(*sets))  # disjoint shares
