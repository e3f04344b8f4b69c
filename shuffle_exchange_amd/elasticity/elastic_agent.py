"""Elastic agent for torchelastic launches (reference elasticity/elastic_agent.py:32 ``DSElasticAgent``,
its monitor loop :127-189).

``SXEElasticAgent`` is a ``LocalElasticAgent`` whose workers get this framework's environment
(rank layout, ``SXE_RESTART_COUNT``, dmabuf IPC for RCCL on ROCm) and whose monitor loop restarts
the worker group on

* a failed / unhealthy worker group -- counted against ``max_restarts``;
* a SHRUNK membership: a node whose rendezvous heartbeat is older than the keep-alive window, or
  fewer participants than the group was started with -- counted against ``max_restarts``;
* GROWN membership (nodes waiting to join) -- not counted: the new world re-rendezvouses, and
  ``elasticity`` recomputes the global batch for the new GPU count at engine start
  (elasticity/elasticity.py ``compute_elastic_config``).

The decision is a pure function (``monitor_decision``) so it is testable without a rendezvous.
The non-torchelastic path is the ``--max_restarts`` option of ``launcher/launch.py`` (same policy,
used by ``bin/sxe``).
"""
import datetime
import logging
import os
import time

try:
    from torch.distributed.elastic.agent.server.api import RunResult, WorkerState
    from torch.distributed.elastic.agent.server.local_elastic_agent import LocalElasticAgent
except Exception:  # pragma: no cover - torch without elastic
    LocalElasticAgent = object
    RunResult = WorkerState = None

log = logging.getLogger(__name__)

SUCCEED, RESTART, RESTART_FREE, FAIL, CONTINUE = "succeed", "restart", "restart_free", "fail", "continue"


def monitor_decision(state, participants_at_start, participants_now, dead_nodes, nodes_waiting, remaining_restarts):
    """One monitor tick: what the agent does next.

    state: "SUCCEEDED" / "HEALTHY" / "UNHEALTHY" / "FAILED" (WorkerState names);
    participants_*: rendezvous participant counts; dead_nodes: nodes past the heartbeat window;
    nodes_waiting: nodes asking to join; remaining_restarts: restarts left.
    """
    if state == "SUCCEEDED":
        return SUCCEED
    shrunk = participants_now < participants_at_start or dead_nodes > 0
    if state in ("UNHEALTHY", "FAILED") or shrunk:
        return RESTART if remaining_restarts > 0 else FAIL
    if state == "HEALTHY":
        return RESTART_FREE if nodes_waiting > 0 else CONTINUE
    raise RuntimeError(f"worker group in unexpected state {state}")


def _rdzv_view(handler, now=None):
    """(participants, dead nodes) from a dynamic rendezvous handler's state holder, defensively: other
    handlers (static / c10d without heartbeats) report what they can."""
    holder = getattr(handler, "_state_holder", None)
    st = getattr(holder, "state", None)
    if st is None:
        return None, 0
    parts = len(getattr(st, "participants", {}) or {})
    settings = getattr(handler, "_settings", None)
    beats = getattr(st, "last_heartbeats", {}) or {}
    dead = 0
    if settings is not None and beats:
        if now is None:
            # torch's dynamic rendezvous stores aware UTC heartbeats (datetime.now(timezone.utc)); match
            # whatever the stored values are so the comparison never mixes naive and aware times
            sample = next(iter(beats.values()))
            now = (datetime.datetime.now(datetime.timezone.utc) if getattr(sample, "tzinfo", None) is not None
                   else datetime.datetime.utcnow())
        window = settings.keep_alive_interval * settings.keep_alive_max_attempt
        dead = sum(1 for t in beats.values() if t < now - window)
    return parts, dead


class SXEElasticAgent(LocalElasticAgent):
    def __init__(self, spec, logs_specs=None, env=None, start_method="spawn", exit_barrier_timeout=300, **kw):
        self.sxe_env = dict(env or {})
        self.sxe_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if logs_specs is None:
            from torch.distributed.elastic.multiprocessing import DefaultLogsSpecs
            logs_specs = DefaultLogsSpecs()
        super().__init__(spec, logs_specs=logs_specs, start_method=start_method,
                         exit_barrier_timeout=exit_barrier_timeout, **kw)

    def _start_workers(self, worker_group):
        for k, v in self.sxe_env.items():
            os.environ.setdefault(k, v)
        os.environ["SXE_RESTART_COUNT"] = str(worker_group.spec.max_restarts - self._remaining_restarts)
        return super()._start_workers(worker_group)

    def _invoke_run(self, role="default"):
        spec = self._worker_group.spec
        role = spec.role
        self._initialize_workers(self._worker_group)
        handler = spec.rdzv_handler
        start_parts, _ = _rdzv_view(handler)
        while True:
            time.sleep(spec.monitor_interval)
            run_result = self._monitor_workers(self._worker_group)
            self._worker_group.state = run_result.state
            parts, dead = _rdzv_view(handler)
            waiting = handler.num_nodes_waiting() if hasattr(handler, "num_nodes_waiting") else 0
            act = monitor_decision(run_result.state.name, start_parts or 0,
                                   parts if parts is not None else (start_parts or 0), dead, waiting,
                                   self._remaining_restarts)
            if act == SUCCEED:
                self._exit_barrier()
                return run_result
            if act == RESTART:
                log.info(f"[{role}] worker group {run_result.state.name} (participants {parts}/{start_parts}, "
                         f"{dead} dead): {self._remaining_restarts}/{spec.max_restarts} restarts left, restarting")
                self._remaining_restarts -= 1
                self._restart_workers(self._worker_group)
                start_parts, _ = _rdzv_view(handler)
            elif act == RESTART_FREE:
                log.info(f"[{role}] {waiting} node(s) waiting to join: restarting the worker group (not counted)")
                self._restart_workers(self._worker_group)
                start_parts, _ = _rdzv_view(handler)
            elif act == FAIL:
                # a shrunk-but-HEALTHY group must still report FAILED, or elastic_launch exits 0 on a job it
                # just killed; like torch's own loop, a failure skips the exit barrier
                self._stop_workers(self._worker_group)
                self._worker_group.state = WorkerState.FAILED
                return RunResult(state=WorkerState.FAILED, failures=dict(run_result.failures or {}))
