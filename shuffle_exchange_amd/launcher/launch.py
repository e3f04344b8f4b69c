"""Per-node launcher: spawns one process per selected local GPU with the torch.distributed env.

Parity: reference launcher/launch.py -- world-info decode, global rank assignment across nodes,
``RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_SIZE / MASTER_ADDR / MASTER_PORT`` per child, per-rank log
files, core binding (``--bind_cores_to_rank``, utils/numa.py), and tearing every child down when
one fails (sigkill_handler) so a crashed rank never leaves the node wedged.

Children are started with ``subprocess.Popen`` before anything here touches the GPU (this process
never initialises HIP), and selected GPUs are exported through ``HIP_VISIBLE_DEVICES``.
"""
import argparse
import os
import signal
import subprocess
import sys
import time

from .runner import decode_world_info


def parse_args(args=None):
    p = argparse.ArgumentParser()
    p.add_argument("--world_info", required=True)
    p.add_argument("--node_rank", type=int, default=0)
    p.add_argument("--master_addr", default="127.0.0.1")
    p.add_argument("--master_port", type=int, default=29500)
    p.add_argument("--module", action="store_true")
    p.add_argument("--no_python", action="store_true")
    p.add_argument("--no_local_rank", action="store_true")
    p.add_argument("--enable_each_rank_log", default="None")
    p.add_argument("--bind_cores_to_rank", action="store_true")
    p.add_argument("--bind_core_list", default=None)
    p.add_argument("--max_restarts", type=int, default=0)
    p.add_argument("user_script")
    p.add_argument("user_args", nargs=argparse.REMAINDER)
    return p.parse_args(args)


def _core_list(rank_local, nlocal, core_list=None):
    if core_list:
        cores = []
        for part in core_list.split(","):
            if "-" in part:
                a, b = part.split("-")
                cores.extend(range(int(a), int(b) + 1))
            else:
                cores.append(int(part))
    else:
        cores = sorted(os.sched_getaffinity(0))
    per = max(1, len(cores) // nlocal)
    return cores[rank_local * per:(rank_local + 1) * per]


def main(args=None):
    """Run the local worker group; on a failure tear it down and, while restarts remain, start a
    fresh group (the reference's DSElasticAgent restart policy, elasticity/elastic_agent.py:127-145).
    Workers see ``SXE_RESTART_COUNT`` (= torchelastic's TORCHELASTIC_RESTART_COUNT) and resume from
    their last checkpoint."""
    a = parse_args(args)
    rc = 0
    for attempt in range(a.max_restarts + 1):
        rc = _run_group(a, attempt)
        if rc == 0:
            return 0
        if attempt < a.max_restarts:
            sys.stderr.write(f"[sxe launch] worker group failed (rc={rc}); restart {attempt + 1}/{a.max_restarts}\n")
    return rc


def _run_group(a, attempt):
    world = decode_world_info(a.world_info)
    hosts = list(world.keys())
    gpus_per_node = [len(world[h]) for h in hosts]
    local = world[hosts[a.node_rank]]
    world_size = sum(gpus_per_node)
    base_rank = sum(gpus_per_node[:a.node_rank])
    procs = []
    env_base = os.environ.copy()
    env_base.update(MASTER_ADDR=a.master_addr, MASTER_PORT=str(a.master_port + attempt), WORLD_SIZE=str(world_size),
                    LOCAL_SIZE=str(len(local)), CROSS_SIZE=str(len(hosts)), CROSS_RANK=str(a.node_rank),
                    SXE_RESTART_COUNT=str(attempt), TORCHELASTIC_RESTART_COUNT=str(attempt))
    env_base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if "HIP_VISIBLE_DEVICES" not in env_base:
        env_base["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in local)

    def kill_all(signum=None, frame=None):
        for p in procs:
            if p.poll() is None:
                try:
                    p.kill()
                except Exception:
                    pass
        if signum is not None:
            sys.exit(128 + signum)

    signal.signal(signal.SIGINT, kill_all)
    signal.signal(signal.SIGTERM, kill_all)
    for lr in range(len(local)):
        env = dict(env_base, RANK=str(base_rank + lr), LOCAL_RANK=str(lr))
        if a.no_python:
            cmd = [a.user_script]
        elif a.module:
            cmd = [sys.executable, "-u", "-m", a.user_script]
        else:
            cmd = [sys.executable, "-u", a.user_script]
        if not a.no_local_rank:
            cmd.append(f"--local_rank={lr}")
        cmd += list(a.user_args)
        if a.bind_cores_to_rank:
            cores = _core_list(lr, len(local), a.bind_core_list)
            env["OMP_NUM_THREADS"] = str(len(cores))
            cmd = ["taskset", "-c", ",".join(map(str, cores))] + cmd
        out = None
        if a.enable_each_rank_log != "None":
            os.makedirs(a.enable_each_rank_log, exist_ok=True)
            out = open(os.path.join(a.enable_each_rank_log, f"rank{base_rank + lr}.log"), "w")
        procs.append(subprocess.Popen(cmd, env=env, stdout=out, stderr=subprocess.STDOUT if out else None))
    rc = 0
    alive = set(range(len(procs)))
    while alive:
        for i in list(alive):
            r = procs[i].poll()
            if r is None:
                continue
            alive.discard(i)
            if r != 0:
                rc = r
                kill_all()
                alive.clear()
                break
        time.sleep(0.1)
    return rc


if __name__ == "__main__":
    sys.exit(main())
