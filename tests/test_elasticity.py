"""Elastic batch-size selection (elasticity/elasticity.py) pinned to hand-derived results of the
reference algorithm (deepspeed/elasticity/elasticity.py): highly-composite-number candidates per
micro batch and per lcm, most valid GPU counts wins, v0.2 node-level search."""
import pytest

from shuffle_exchange_amd.elasticity import (ElasticityConfigError, ElasticityIncompatibleWorldSize,
                                             compute_elastic_config)
from shuffle_exchange_amd.elasticity.elasticity import candidate_batch_sizes, valid_gpus


def _cfg(**kw):
    el = {"enabled": True, "max_train_batch_size": 2000, "micro_batch_sizes": [2, 4, 6], "min_gpus": 1,
          "max_gpus": 10000, "version": 0.1}
    el.update(kw)
    return {"elasticity": el}


def _divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def test_v01_candidates_and_choice():
    # bases 2, 4, 6 and lcm 12 scaled by the largest HCN <= 2000 // base: 840*2, 360*4, 240*6, 120*12
    assert candidate_batch_sizes([2, 4, 6], 2000) == [1440, 1680]
    # 1440 is valid for the 30 divisors of 720, 1680 for the 32 divisors of 840
    assert valid_gpus(1440, [2, 4, 6], 1, 10000) == _divisors(720)
    batch, gpus = compute_elastic_config(_cfg())
    assert batch == 1680 and gpus == _divisors(840)
    for g in gpus:
        assert batch % g == 0 and any((batch // g) % m == 0 for m in (2, 4, 6))


def test_v01_world_size_micro_batch_and_rejection():
    b, gpus, mb = compute_elastic_config(_cfg(), world_size=7)
    assert (b, mb) == (1680, 6)  # 1680 // 7 = 240: the largest listed micro batch dividing it
    b, gpus, mb = compute_elastic_config(_cfg(), world_size=42)
    assert mb == 4  # 1680 // 42 = 40
    with pytest.raises(ElasticityIncompatibleWorldSize):
        compute_elastic_config(_cfg(), world_size=9)


def test_v01_gpu_range_and_cap():
    # in [100, 500]: 1440 has 5 valid counts (divisors of 720), 1680 has 7 (divisors of 840)
    b, gpus = compute_elastic_config(_cfg(min_gpus=100, max_gpus=500))
    assert b == 1680 and gpus == [105, 120, 140, 168, 210, 280, 420]
    # a micro batch at the cap is its own candidate
    assert candidate_batch_sizes([64], 64) == [64]
    with pytest.raises(ElasticityConfigError):
        compute_elastic_config(_cfg(micro_batch_sizes=[4096]))
    with pytest.raises(ElasticityConfigError):
        compute_elastic_config(_cfg(model_parallel_size=2))  # model parallel needs v0.2
    with pytest.raises(ElasticityConfigError):
        compute_elastic_config(_cfg(enabled=False))


def test_v02_node_level_search():
    cfg = _cfg(max_train_batch_size=1024, micro_batch_sizes=[2, 4], min_gpus=8, max_gpus=64,
               model_parallel_size=2, num_gpus_per_node=8, version=0.2)
    # per node: 4 data-parallel ranks, batch cap 1024 / 4 = 256 -> candidates 120*2 = 60*4 = 240,
    # valid for 1..8 nodes dividing 120 -> data-parallel sizes 4 * {1, 2, 3, 4, 5, 6, 8}
    b, valid, mb = compute_elastic_config(cfg, world_size=16)
    assert b == 960 and valid == [4, 8, 12, 16, 20, 24, 32] and mb == 4
    with pytest.raises(ElasticityConfigError):
        compute_elastic_config(dict(elasticity=dict(cfg["elasticity"], num_gpus_per_node=5)), world_size=16)


def test_v02_world_size_from_env(monkeypatch):
    cfg = _cfg(max_train_batch_size=1024, micro_batch_sizes=[2, 4], min_gpus=8, max_gpus=64,
               model_parallel_size=2, num_gpus_per_node=8, version=0.2)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(ElasticityConfigError):
        compute_elastic_config(cfg)
    monkeypatch.setenv("WORLD_SIZE", "16")
    b, valid, mb = compute_elastic_config(cfg, return_microbatch=True)
    assert (b, mb) == (960, 4)


def test_elastic_agent_monitor_decisions():
    """The agent's monitor tick (reference elasticity/elastic_agent.py:127-189): failures and shrunk
    membership (dead heartbeat / fewer participants) restart against max_restarts, grown membership
    restarts for free, success exits."""
    from shuffle_exchange_amd.elasticity.elastic_agent import (FAIL, RESTART, RESTART_FREE, SUCCEED, CONTINUE,
                                                               monitor_decision)
    assert monitor_decision("SUCCEEDED", 2, 2, 0, 0, 3) == SUCCEED
    assert monitor_decision("HEALTHY", 2, 2, 0, 0, 3) == CONTINUE
    assert monitor_decision("HEALTHY", 2, 2, 0, 1, 0) == RESTART_FREE     # joiners: not counted
    assert monitor_decision("FAILED", 2, 2, 0, 0, 1) == RESTART
    assert monitor_decision("UNHEALTHY", 2, 2, 0, 0, 0) == FAIL
    assert monitor_decision("HEALTHY", 3, 2, 0, 0, 1) == RESTART          # a participant left
    assert monitor_decision("HEALTHY", 2, 2, 1, 0, 1) == RESTART          # a dead heartbeat
    assert monitor_decision("HEALTHY", 2, 2, 1, 0, 0) == FAIL


def test_elastic_agent_rdzv_view_counts_dead_heartbeats():
    import datetime
    import types
    from shuffle_exchange_amd.elasticity.elastic_agent import _rdzv_view
    now = datetime.datetime(2026, 1, 1, 12, 0, 0)
    st = types.SimpleNamespace(participants={"a": 0, "b": 1},
                               last_heartbeats={"a": now, "b": now - datetime.timedelta(seconds=100)})
    h = types.SimpleNamespace(_state_holder=types.SimpleNamespace(state=st),
                              _settings=types.SimpleNamespace(keep_alive_interval=datetime.timedelta(seconds=5),
                                                              keep_alive_max_attempt=3))
    assert _rdzv_view(h, now) == (2, 1)
    assert _rdzv_view(types.SimpleNamespace()) == (None, 0)


def test_elastic_agent_rdzv_view_aware_heartbeats_default_now():
    """torch's DynamicRendezvousHandler stores aware UTC heartbeats; the default ``now`` must compare
    against them without a naive/aware TypeError."""
    import datetime
    import types
    from shuffle_exchange_amd.elasticity.elastic_agent import _rdzv_view
    now = datetime.datetime.now(datetime.timezone.utc)
    st = types.SimpleNamespace(participants={"a": 0, "b": 1, "c": 2},
                               last_heartbeats={"a": now, "b": now - datetime.timedelta(seconds=100),
                                                "c": now - datetime.timedelta(seconds=1)})
    h = types.SimpleNamespace(_state_holder=types.SimpleNamespace(state=st),
                              _settings=types.SimpleNamespace(keep_alive_interval=datetime.timedelta(seconds=5),
                                                              keep_alive_max_attempt=3))
    assert _rdzv_view(h) == (3, 1)


def test_elastic_agent_fail_on_shrunk_healthy_group_reports_failed():
    """Membership shrank, the local group is still HEALTHY, no restarts left: the agent stops the
    workers and returns a FAILED result (so elastic_launch exits non-zero) without the exit barrier."""
    import datetime
    import types
    from torch.distributed.elastic.agent.server.api import RunResult, WorkerState
    from shuffle_exchange_amd.elasticity.elastic_agent import SXEElasticAgent
    now = datetime.datetime.now(datetime.timezone.utc)
    beats = {"a": now, "b": now}
    st = types.SimpleNamespace(participants={"a": 0, "b": 1}, last_heartbeats=beats)
    handler = types.SimpleNamespace(_state_holder=types.SimpleNamespace(state=st),
                                    _settings=types.SimpleNamespace(keep_alive_interval=datetime.timedelta(seconds=5),
                                                                    keep_alive_max_attempt=3),
                                    num_nodes_waiting=lambda: 0)
    calls = []

    class Fake:
        _remaining_restarts = 0
        _worker_group = types.SimpleNamespace(spec=types.SimpleNamespace(role="default", rdzv_handler=handler,
                                                                         monitor_interval=0, max_restarts=0),
                                              state=None)

        def _initialize_workers(self, wg):
            calls.append("init")

        def _monitor_workers(self, wg):
            beats["b"] = now - datetime.timedelta(seconds=100)       # node b stops heart-beating
            return RunResult(state=WorkerState.HEALTHY)

        def _stop_workers(self, wg):
            calls.append("stop")

        def _exit_barrier(self):
            calls.append("barrier")

    res = SXEElasticAgent._invoke_run(Fake())
    assert res.state == WorkerState.FAILED and res.is_failed()
    assert calls == ["init", "stop"]
    assert Fake._worker_group.state == WorkerState.FAILED
