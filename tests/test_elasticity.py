"""Elastic batch-size selection: every reported GPU count divides the batch with a listed micro
batch; incompatible world sizes are rejected; micro batch returned for a given world size."""
import pytest


def test_compute_elastic_config():
    from shuffle_exchange_amd.elasticity import ElasticityIncompatibleWorldSize, compute_elastic_config
    cfg = {"elasticity": {"enabled": True, "max_train_batch_size": 2000, "micro_batch_sizes": [2, 4, 6],
                          "min_gpus": 1, "max_gpus": 64, "version": 0.1}}
    batch, gpus = compute_elastic_config(cfg)
    assert batch <= 2000 and len(gpus) > 10
    for g in gpus:
        assert batch % g == 0 and any((batch // g) % m == 0 for m in (2, 4, 6))
    b2, g2, mb = compute_elastic_config(cfg, world_size=gpus[-1], return_microbatch=True)
    assert b2 == batch and (batch // gpus[-1]) % mb == 0
    bad = next(g for g in range(1, 65) if g not in gpus)
    with pytest.raises(ElasticityIncompatibleWorldSize):
        compute_elastic_config(cfg, world_size=bad)


def test_elastic_model_parallel():
    from shuffle_exchange_amd.elasticity import compute_elastic_config
    cfg = {"elasticity": {"enabled": True, "max_train_batch_size": 1024, "micro_batch_sizes": [1, 2, 4],
                          "min_gpus": 8, "max_gpus": 64, "model_parallel_size": 8, "num_gpus_per_node": 8,
                          "version": 0.2}}
    batch, gpus = compute_elastic_config(cfg)
    assert all(g % 8 == 0 for g in gpus)
