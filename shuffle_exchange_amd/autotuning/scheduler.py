"""Experiment scheduler for the autotuner (reference autotuning/scheduler.py ``ResourceManager`` :32):
runs queued experiments on the node's GPUs, as many at once as their GPU counts allow, each in its
own process group with its own device set, config, logs and metric file, and parses the results.

An experiment directory ``exps_dir/<name>/`` holds ``ds_config.json``, ``cmd.txt``,
``stdout.log`` / ``stderr.log`` and the ``metrics.json`` the engine writes between
``start_profile_step`` and ``end_profile_step`` (runtime/engine.py ``_autotuning_probe``).
Devices are handed out with ``HIP_VISIBLE_DEVICES`` (one process per GPU inside an experiment,
rendezvous on 127.0.0.1 with a port per experiment). Only the local node is scheduled: a multi-node
search would launch through the regular launcher (launcher/runner.py) with a hostfile per
experiment, which the reference does over pdsh.
"""
import json
import os
import signal
import subprocess
import sys
import time

from ..utils.logging import logger


class Experiment:
    def __init__(self, name, ds_config, num_gpus=1, overrides=None):
        self.name = name
        self.ds_config = ds_config
        self.num_gpus = int(num_gpus)
        self.overrides = overrides or {}
        self.metrics = None
        self.error = None
        self.secs = None

    @property
    def metric(self):
        return None if self.metrics is None else self.metrics.get("_selected")

    def __repr__(self):
        return f"Experiment({self.name}, metric={self.metric})"


class ResourceManager:
    def __init__(self, user_script, user_args=(), num_gpus=1, exps_dir="autotuning_exps", metric="throughput",
                 exp_timeout=1800, start_profile_step=3, end_profile_step=5, poll_s=0.5, base_port=29600,
                 python=sys.executable, use_torchrun=True):
        self.user_script, self.user_args = user_script, list(user_args)
        self.num_gpus = int(num_gpus)
        self.exps_dir = exps_dir
        self.metric = metric
        self.exp_timeout = exp_timeout
        self.profile = (start_profile_step, end_profile_step)
        self.poll_s = poll_s
        self.base_port = base_port
        self.python = python
        self.use_torchrun = use_torchrun
        self.queue, self.finished = [], []
        self._free = list(range(self.num_gpus))
        self._port = 0

    # -------------------------------------------------------------------------------- queueing
    def schedule_experiments(self, exps):
        for e in exps:
            assert 1 <= e.num_gpus <= self.num_gpus, f"{e.name}: needs {e.num_gpus} GPUs, node has {self.num_gpus}"
            self.queue.append(e)

    def _next_port(self):
        self._port += 1
        return self.base_port + self._port % 1000

    def _command(self, exp, cfg_path):
        if self.use_torchrun:
            return [self.python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={exp.num_gpus}",
                    "--master-addr", "127.0.0.1", "--master-port", str(self._next_port()),
                    self.user_script, "--deepspeed_config", cfg_path] + self.user_args
        return [self.python, self.user_script, "--deepspeed_config", cfg_path] + self.user_args

    def _start(self, exp):
        d = os.path.abspath(os.path.join(self.exps_dir, exp.name))
        os.makedirs(d, exist_ok=True)
        mpath = os.path.join(d, "metrics.json")
        if os.path.exists(mpath):
            os.remove(mpath)
        cfg = json.loads(json.dumps(exp.ds_config))
        at = dict(cfg.get("autotuning", {}))
        at.update({"enabled": True, "metric_path": mpath, "start_profile_step": self.profile[0],
                   "end_profile_step": self.profile[1], "exit_after_profile": True})
        cfg["autotuning"] = at
        cfg_path = os.path.join(d, "ds_config.json")
        with open(cfg_path, "w") as f:
            json.dump(cfg, f, indent=2)
        devs = [self._free.pop(0) for _ in range(exp.num_gpus)]
        cmd = self._command(exp, cfg_path)
        with open(os.path.join(d, "cmd.txt"), "w") as f:
            f.write(" ".join(cmd) + "\n")
        env = dict(os.environ)
        env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, devs))
        if not self.use_torchrun:  # single-process experiment: its own rendezvous
            assert exp.num_gpus == 1, "multi-GPU experiments need use_torchrun=True"
            env.update({"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "LOCAL_WORLD_SIZE": "1",
                        "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(self._next_port())})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        out, err = open(os.path.join(d, "stdout.log"), "w"), open(os.path.join(d, "stderr.log"), "w")
        proc = subprocess.Popen(cmd, stdout=out, stderr=err, env=env, start_new_session=True)
        return {"exp": exp, "proc": proc, "devs": devs, "t0": time.time(), "mpath": mpath, "files": (out, err)}

    def _finish(self, r, rc):
        exp = r["exp"]
        for f in r["files"]:
            f.close()
        self._free.extend(r["devs"])
        self._free.sort()
        exp.secs = time.time() - r["t0"]
        if os.path.exists(r["mpath"]):
            with open(r["mpath"]) as f:
                m = json.load(f)
            m["_selected"] = m.get(self.metric)
            if self.metric == "latency" and m["_selected"] is not None:
                m["_selected"] = -m["_selected"]  # higher is better everywhere in the tuners
            exp.metrics = m
        else:
            exp.error = f"exit code {rc}, no metrics (see {os.path.join(self.exps_dir, exp.name, 'stderr.log')})"
        self.finished.append(exp)
        logger.info(f"autotuning: {exp.name} -> {exp.metrics if exp.metrics else exp.error} ({exp.secs:.1f}s)")

    def run(self):
        """Run every queued experiment; returns them (finished order)."""
        running = []
        done = []
        while self.queue or running:
            i = 0
            while i < len(self.queue):  # first-fit: start whatever the free GPUs allow
                if self.queue[i].num_gpus <= len(self._free):
                    running.append(self._start(self.queue.pop(i)))
                else:
                    i += 1
            time.sleep(self.poll_s)
            for r in list(running):
                rc = r["proc"].poll()
                if rc is None and time.time() - r["t0"] > self.exp_timeout:
                    os.killpg(r["proc"].pid, signal.SIGKILL)  # the experiment's own process group
                    rc = r["proc"].wait()
                    r["exp"].error = "timeout"
                if rc is not None:
                    running.remove(r)
                    self._finish(r, rc)
                    done.append(r["exp"])
        return done

    def parse_results(self):
        ok = [e for e in self.finished if e.metric is not None]
        best = max(ok, key=lambda e: e.metric) if ok else None
        return best

    def run_one(self, exp):
        """Blocking single experiment (the tuners' evaluation callback)."""
        self.schedule_experiments([exp])
        self.run()
        if exp.metrics is None:
            raise RuntimeError(exp.error or "experiment failed")
        return exp.metric
