"""Elastic training: pick a global batch size that stays valid across many GPU counts.

Parity: reference elasticity/elasticity.py -- ``compute_elastic_config`` :233 (v0.1 and v0.2 with
model-parallel size and GPUs per node), ``ElasticityConfig`` keys (max_train_batch_size,
micro_batch_sizes, min_gpus, max_gpus, min_time, version, prefer_larger_batch,
ignore_non_elastic_batch_info, model_parallel_size, num_gpus_per_node) and the
``ElasticityError`` family. ``elastic_agent.py`` (torchelastic agent) maps to launching through
``torch.distributed.run --nnodes=min:max`` with this config; see docs.

A batch size B is valid for G data-parallel ranks when some micro-batch size m in the list divides
B / G (gradient accumulation makes up the rest). Among candidate batches <= max_train_batch_size
(multiples of the micro-batch lcm, plus the largest multiple of every micro batch), the one valid
for the most GPU counts in [min_gpus, max_gpus] wins; ties go to the larger (or smaller) batch.
"""
import math
from functools import reduce

LATEST_ELASTICITY_VERSION = 0.2


class ElasticityError(Exception):
    pass


class ElasticityConfigError(ElasticityError):
    pass


class ElasticityIncompatibleWorldSize(ElasticityError):
    pass


def _lcm(a, b):
    return a * b // math.gcd(a, b)


def _candidate_batches(micro, max_batch):
    base = reduce(_lcm, micro)
    cands = set()
    k = 1
    while base * k <= max_batch:
        cands.add(base * k)
        k += 1
    for m in micro:
        if m <= max_batch:
            cands.add((max_batch // m) * m)
    return sorted(cands)


def _valid_gpus(batch, micro, min_g, max_g):
    out = []
    for g in range(min_g, max_g + 1):
        if batch % g:
            continue
        per = batch // g
        if any(per % m == 0 for m in micro):
            out.append(g)
    return out


def get_best_candidates(micro, max_batch, min_g, max_g, prefer_larger=True):
    best, best_gpus = None, []
    for b in _candidate_batches(micro, max_batch):
        gpus = _valid_gpus(b, micro, min_g, max_g)
        better = len(gpus) > len(best_gpus) or (len(gpus) == len(best_gpus) and gpus and
                                                 ((prefer_larger and b > best) or (not prefer_larger and b < best)))
        if better:
            best, best_gpus = b, gpus
    return best, best_gpus


def compute_elastic_config(ds_config, target_deepspeed_version=None, world_size=0, return_microbatch=False):
    """Returns (final_batch_size, valid_gpus) or (final_batch_size, valid_gpus, micro_batch_size)."""
    el = ds_config.get("elasticity", ds_config) if isinstance(ds_config, dict) else ds_config
    get = (lambda k, d=None: el.get(k, d)) if isinstance(el, dict) else (lambda k, d=None: getattr(el, k, d))
    if isinstance(el, dict) and not el.get("enabled", True):
        raise ElasticityConfigError("elasticity is not enabled")
    micro = sorted(set(int(m) for m in get("micro_batch_sizes", [])))
    if not micro or any(m <= 0 for m in micro):
        raise ElasticityConfigError("micro_batch_sizes must be a non-empty list of positive ints")
    max_batch = int(get("max_train_batch_size", 0))
    if max_batch <= 0:
        raise ElasticityConfigError("max_train_batch_size must be positive")
    min_g, max_g = int(get("min_gpus", 1)), int(get("max_gpus", 10000))
    if min_g < 1 or max_g < min_g:
        raise ElasticityConfigError("need 1 <= min_gpus <= max_gpus")
    version = float(get("version", LATEST_ELASTICITY_VERSION))
    prefer_larger = bool(get("prefer_larger_batch", True))
    mp = int(get("model_parallel_size", 1)) if version >= 0.2 else 1
    gpn = int(get("num_gpus_per_node", 1)) if version >= 0.2 else 1
    if mp > 1 and gpn % mp and mp % gpn:
        raise ElasticityConfigError("model_parallel_size and num_gpus_per_node must divide one another")
    # data-parallel ranks = GPUs / mp; whole nodes only when mp spans nodes
    dmin, dmax = max(1, math.ceil(min_g / mp)), max(1, max_g // mp)
    batch, dp_counts = get_best_candidates(micro, max_batch, dmin, dmax, prefer_larger)
    if batch is None or not dp_counts:
        raise ElasticityError(f"no valid batch size <= {max_batch} for micro batches {micro}")
    valid_gpus = [d * mp for d in dp_counts if (d * mp) % max(1, min(gpn, d * mp)) == 0 or mp == 1]
    if world_size > 0 and world_size not in valid_gpus:
        raise ElasticityIncompatibleWorldSize(f"world size {world_size} is not in the valid set {valid_gpus}")
    if return_microbatch:
        dp = (world_size // mp) if world_size > 0 else dp_counts[0]
        per = batch // dp
        mb = max(m for m in micro if per % m == 0)
        return batch, valid_gpus, mb
    return batch, valid_gpus


def elasticity_enabled(ds_config):
    return bool(ds_config.get("elasticity", {}).get("enabled", False)) if isinstance(ds_config, dict) else False
