"""Elastic agent for torchelastic launches (reference elasticity/elastic_agent.py:32 ``DSElasticAgent``).

``SXEElasticAgent`` is a ``LocalElasticAgent`` whose workers get this framework's environment
(rank layout, ``SXE_RESTART_COUNT``, dmabuf IPC for RCCL on ROCm) and whose worker group is
restarted on failure / membership change up to ``max_restarts`` (torchelastic's policy, which the
reference also relies on). The non-torchelastic path is the ``--max_restarts`` option of
``launcher/launch.py`` (same policy, used by ``bin/sxe``).
"""
import os

try:
    from torch.distributed.elastic.agent.server.local_elastic_agent import LocalElasticAgent
except Exception:  # pragma: no cover - torch without elastic
    LocalElasticAgent = object


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
