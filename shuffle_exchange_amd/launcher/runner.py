"""``sxe`` launcher: resource discovery (hostfile / include / exclude), then one ``launch`` per node
via ssh-style multi-node runners or directly on this node.

Parity: reference launcher/runner.py -- ``parse_args`` :48, ``fetch_hostfile`` / ``_parse_hostfile``
:213-265, ``parse_resource_filter`` :275-350 (``host1:0,1@host2`` syntax), ``parse_inclusion_exclusion``,
``encode_world_info`` :376, ``main`` :430-636 (PDSH / OpenMPI / MPICH / Slurm runners,
``.deepspeed_env`` export). MI355X default: 8 GPUs per node (``rocm-smi``-free discovery through
``torch.cuda.device_count()`` which does not initialise HIP), RCCL over xGMI inside the node.
"""
import argparse
import base64
import collections
import json
import os
import shlex
import subprocess
import sys

DEFAULT_HOSTFILE = "/job/hostfile"
ENV_FILES = (".sxe_env", ".deepspeed_env")
EXPORT_ENVS = ("NCCL", "RCCL", "HSA", "HIP", "ROCM", "PYTHON", "MIOPEN", "OMP", "SXE", "TORCH", "UCX")


def parse_args(args=None):
    p = argparse.ArgumentParser(description="sxe distributed launcher (one process per MI355X GPU)")
    p.add_argument("-H", "--hostfile", default=DEFAULT_HOSTFILE)
    p.add_argument("-i", "--include", default="")
    p.add_argument("-e", "--exclude", default="")
    p.add_argument("--num_nodes", type=int, default=-1)
    p.add_argument("--min_elastic_nodes", type=int, default=-1)
    p.add_argument("--max_elastic_nodes", type=int, default=-1)
    p.add_argument("--num_gpus", "--num_accelerators", type=int, default=-1, dest="num_gpus")
    p.add_argument("--master_port", type=int, default=29500)
    p.add_argument("--master_addr", default="")
    p.add_argument("--launcher", default="pdsh", choices=["pdsh", "openmpi", "mpich", "slurm", "ssh", "local"])
    p.add_argument("--launcher_args", default="")
    p.add_argument("--module", action="store_true")
    p.add_argument("--no_python", action="store_true")
    p.add_argument("--no_local_rank", action="store_true")
    p.add_argument("--no_ssh_check", action="store_true")
    p.add_argument("--force_multi", action="store_true")
    p.add_argument("--save_pid", action="store_true")
    p.add_argument("--enable_each_rank_log", default="None")
    p.add_argument("--bind_cores_to_rank", action="store_true")
    p.add_argument("--bind_core_list", default=None)
    p.add_argument("--elastic_training", action="store_true")
    p.add_argument("--max_restarts", type=int, default=0,
                   help="restart the local worker group up to N times after a failure (elastic agent)")
    p.add_argument("--dry_run", action="store_true", help="print the per-node commands and exit")
    p.add_argument("--autotuning", default="", choices=["", "tune", "run"],
                   help="tune: search ZeRO stage x micro batch with short runs; run: tune then launch the best")
    p.add_argument("user_script")
    p.add_argument("user_args", nargs=argparse.REMAINDER)
    return p.parse_args(args)


def parse_hostfile(lines):
    """``hostname slots=N`` per line (comments with #) -> OrderedDict host -> slots."""
    pool = collections.OrderedDict()
    for raw in lines:
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        parts = line.split()
        host = parts[0]
        slots = None
        for tok in parts[1:]:
            if tok.startswith("slots="):
                slots = int(tok.split("=", 1)[1])
        if slots is None:
            raise ValueError(f"hostfile line without slots=: {raw!r}")
        if host in pool:
            raise ValueError(f"host {host} listed twice in hostfile")
        pool[host] = slots
    return pool


def fetch_hostfile(path):
    if not path or not os.path.isfile(path):
        return None
    with open(path) as f:
        return parse_hostfile(f.readlines())


def _parse_filter(s):
    """``host1:0,1@host2`` -> {host1: [0, 1], host2: None (all)}."""
    out = collections.OrderedDict()
    if not s:
        return out
    for item in s.split("@"):
        item = item.strip()
        if not item:
            continue
        if ":" in item:
            host, slots = item.split(":", 1)
            out[host] = [int(x) for x in slots.split(",") if x != ""]
        else:
            out[item] = None
    return out


def parse_resource_filter(host_info, include_str="", exclude_str=""):
    """Apply include / exclude to {host: slot count} -> {host: [gpu ids]}."""
    if include_str and exclude_str:
        raise ValueError("include and exclude are mutually exclusive")
    full = collections.OrderedDict((h, list(range(n))) for h, n in host_info.items())
    if include_str:
        inc = _parse_filter(include_str)
        out = collections.OrderedDict()
        for h, slots in inc.items():
            if h not in full:
                raise ValueError(f"included host {h} not in hostfile")
            sel = full[h] if slots is None else slots
            for s_ in sel:
                if s_ not in full[h]:
                    raise ValueError(f"host {h} has no slot {s_}")
            out[h] = sorted(sel)
        return out
    if exclude_str:
        exc = _parse_filter(exclude_str)
        out = collections.OrderedDict()
        for h, slots in full.items():
            if h in exc:
                if exc[h] is None:
                    continue
                keep = [s_ for s_ in slots if s_ not in exc[h]]
                if keep:
                    out[h] = keep
            else:
                out[h] = slots
        return out
    return full


def encode_world_info(world_info):
    return base64.urlsafe_b64encode(json.dumps(world_info).encode()).decode()


def decode_world_info(s):
    return json.loads(base64.urlsafe_b64decode(s.encode()).decode())


def _local_gpu_count():
    try:
        import torch
        return max(1, torch.cuda.device_count())
    except Exception:
        return 1


def _exports():
    env = {}
    for k, v in os.environ.items():
        if any(k.startswith(p) for p in EXPORT_ENVS):
            env[k] = v
    for fn in ENV_FILES:
        for d in (os.path.expanduser("~"), os.getcwd()):
            path = os.path.join(d, fn)
            if os.path.isfile(path):
                with open(path) as f:
                    for line in f:
                        line = line.strip()
                        if line and "=" in line and not line.startswith("#"):
                            k, v = line.split("=", 1)
                            env[k] = v
    return env


def build_launch_cmd(args, world_info_b64, node_rank, master_addr):
    cmd = [sys.executable, "-u", "-m", "shuffle_exchange_amd.launcher.launch", f"--world_info={world_info_b64}",
           f"--node_rank={node_rank}", f"--master_addr={master_addr}", f"--master_port={args.master_port}"]
    if args.module:
        cmd.append("--module")
    if args.no_python:
        cmd.append("--no_python")
    if args.no_local_rank:
        cmd.append("--no_local_rank")
    if args.bind_cores_to_rank:
        cmd.append("--bind_cores_to_rank")
        if args.bind_core_list:
            cmd.append(f"--bind_core_list={args.bind_core_list}")
    if args.enable_each_rank_log != "None":
        cmd.append(f"--enable_each_rank_log={args.enable_each_rank_log}")
    if getattr(args, "max_restarts", 0):
        cmd.append(f"--max_restarts={args.max_restarts}")
    return cmd + [args.user_script] + list(args.user_args)


def multinode_commands(args, active, master_addr):
    """One remote command per node for the chosen runner (pdsh/ssh/openmpi/mpich/slurm)."""
    wi = encode_world_info(active)
    exports = " ".join(f"export {k}={shlex.quote(v)};" for k, v in _exports().items())
    cmds = []
    for node_rank, host in enumerate(active):
        inner = " ".join(shlex.quote(c) for c in build_launch_cmd(args, wi, node_rank, master_addr))
        remote = f"cd {shlex.quote(os.path.abspath('.'))}; {exports} {inner}"
        if args.launcher in ("pdsh", "ssh"):
            cmds.append(["ssh", host, remote] if args.launcher == "ssh" else ["pdsh", "-S", "-f", "1024", "-w", host,
                                                                              remote])
        elif args.launcher == "slurm":
            cmds.append(["srun", "-N", "1", "-w", host] + shlex.split(args.launcher_args) + ["bash", "-c", remote])
        else:  # openmpi / mpich: one mpirun for all nodes is typical; per-node form keeps it uniform
            cmds.append(["mpirun", "-n", "1", "-host", host] + shlex.split(args.launcher_args) + ["bash", "-c", remote])
    return cmds


def _autotune(args):
    import json
    from ..autotuning import Autotuner, scheduled_runner
    ua = list(args.user_args)
    cfg_path = None
    for i, a in enumerate(ua):
        if a in ("--deepspeed_config", "--sxe_config") and i + 1 < len(ua):
            cfg_path = ua[i + 1]
            rest = ua[:i] + ua[i + 2:]
            break
    else:
        raise SystemExit("--autotuning needs --deepspeed_config <json> in the user arguments")
    with open(cfg_path) as f:
        base = json.load(f)
    at_cfg = base.get("autotuning", {})
    nproc = args.num_gpus if args.num_gpus > 0 else _local_gpu_count()
    tuner = Autotuner(base, world_size=nproc)
    run = scheduled_runner(args.user_script, rest, exps_dir=tuner.exps_dir, nproc=nproc,
                           timeout=tuner.at.exp_timeout, start_step=tuner.at.start_profile_step,
                           end_step=tuner.at.end_profile_step, metric=tuner.metric)
    best = tuner.tune(run, profile_model_info=not tuner.model_info.get("num_params"))
    best_cfg = tuner.best_config()
    if best_cfg is not None:
        tuner.write_optimal_cmd(args.user_script, rest)
    print(f"autotuning best: {best}")
    if args.autotuning == "run" and best_cfg is not None:
        best_cfg.pop("autotuning", None)
        out = os.path.join(tuner.results_dir, "best_config.json")
        with open(out, "w") as f:
            json.dump(best_cfg, f, indent=2)
        args.user_args = rest + ["--deepspeed_config", out]
        args.autotuning = ""
        return main_with(args)
    return 0


def main(args=None):
    args = parse_args(args)
    if args.autotuning:
        return _autotune(args)
    return main_with(args)


def main_with(args):
    pool = fetch_hostfile(args.hostfile)
    if pool is None:
        n = args.num_gpus if args.num_gpus > 0 else _local_gpu_count()
        pool = collections.OrderedDict(localhost=n)
        multi = False
    else:
        multi = True
    active = parse_resource_filter(pool, args.include, args.exclude)
    if args.num_nodes > 0:
        active = collections.OrderedDict(list(active.items())[:args.num_nodes])
    if args.num_gpus > 0:
        active = collections.OrderedDict((h, s[:args.num_gpus]) for h, s in active.items())
    if not active:
        raise RuntimeError("no resources selected")
    master_addr = args.master_addr or ("127.0.0.1" if not multi or len(active) == 1 else next(iter(active)))
    if len(active) == 1 and not args.force_multi:
        wi = encode_world_info(active)
        cmd = build_launch_cmd(args, wi, 0, master_addr)
        if args.dry_run:
            print(" ".join(shlex.quote(c) for c in cmd))
            return 0
        return subprocess.call(cmd, env=os.environ.copy())
    cmds = multinode_commands(args, active, master_addr)
    if args.dry_run:
        for c in cmds:
            print(" ".join(shlex.quote(x) for x in c))
        return 0
    procs = [subprocess.Popen(c) for c in cmds]
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
