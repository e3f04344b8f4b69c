"""Elastic training: pick a global batch size that stays valid across many GPU counts.

Parity: reference elasticity/elasticity.py -- ``compute_elastic_config`` :233 (v0.1 and v0.2 with
model-parallel size and GPUs per node), ``ElasticityConfig`` keys (max_train_batch_size,
micro_batch_sizes, min_gpus, max_gpus, min_time, version, prefer_larger_batch,
ignore_non_elastic_batch_info, model_parallel_size, num_gpus_per_node) and the
``ElasticityError`` family. ``elastic_agent.py`` (torchelastic agent) maps to launching through
``torch.distributed.run --nnodes=min:max`` with this config; see docs.

A batch size B is valid for G data-parallel ranks when some micro-batch size m in the list divides
B / G (gradient accumulation makes up the rest). The candidates are the reference's: for every
micro batch and for their lcm, the base scaled by the largest highly composite number that keeps
it <= max_train_batch_size (a base already at or above the cap is its own candidate). The
candidate valid for the most GPU counts in [min_gpus, max_gpus] wins; ties go to the larger (or
smaller, ``prefer_larger_batch: false``) batch. v0.2 runs the same search per NODE (GPU counts in
whole nodes, batch per data-parallel rank of a node) and, for a world size outside the valid set,
falls back to the largest multiple of (micro batch x current data-parallel size) under the cap.
Given the same config, the results equal the reference's (``tests/test_elasticity.py`` pins
hand-derived cases).
"""
import math
import os
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


# the 38 smallest highly composite numbers (OEIS A002182)
HCN_LIST = [1, 2, 4, 6, 12, 24, 36, 48, 60, 120, 180, 240, 360, 720, 840, 1260, 1680, 2520, 5040, 7560, 10080,
            15120, 20160, 25200, 27720, 45360, 50400, 55440, 83160, 110880, 166320, 221760, 277200, 332640,
            498960, 554400, 665280, 720720]


def _largest_hcn_at_most(v):
    best = HCN_LIST[-1]
    for h in HCN_LIST:
        if h > v:
            break
        best = h
    return best


def candidate_batch_sizes(micro, max_batch):
    bases = list(micro) + [reduce(_lcm, micro)]
    return sorted({b if b >= max_batch else _largest_hcn_at_most(max_batch // b) * b for b in bases})


def valid_gpus(batch, micro, min_g, max_g):
    """GPU counts G in [min_g, max_g] with B % G == 0 and (B / G) % m == 0 for some micro batch m."""
    out = set()
    for m in micro:
        if batch % m:
            continue
        top = batch // m  # G may be any divisor of B / m
        for g in range(max(1, min_g), min(top, max_g) + 1):
            if top % g == 0:
                out.add(g)
    return sorted(out)


def get_best_candidates(micro, max_batch, min_g, max_g, prefer_larger=True):
    best, best_gpus = int(min(micro)), None
    n_best = 0
    for b in candidate_batch_sizes(micro, max_batch):
        gpus = valid_gpus(b, micro, min_g, max_g)
        if len(gpus) > n_best or (len(gpus) == n_best and
                                  ((prefer_larger and b > best) or (not prefer_larger and b < best))):
            best, best_gpus, n_best = b, gpus, len(gpus)
    return best, best_gpus


def _largest_dividing_micro(batch, world, micro, prefer_larger=True):
    fits = [m for m in micro if (batch // world) % m == 0]
    if not fits:
        return None
    return max(fits) if prefer_larger else min(fits)


def compute_elastic_config(ds_config, target_deepspeed_version=None, world_size=0, return_microbatch=False):
    """Returns (final_batch_size, valid_gpus), plus the micro batch size when ``world_size`` is
    given or ``return_microbatch`` (reference elasticity.py:233)."""
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
    if any(m > max_batch for m in micro):
        raise ElasticityConfigError(f"every micro batch must be <= max_train_batch_size ({max_batch})")
    min_g, max_g = int(get("min_gpus", 1)), int(get("max_gpus", 10000))
    if min_g < 1 or max_g < min_g:
        raise ElasticityConfigError("need 1 <= min_gpus <= max_gpus")
    version = float(get("version", LATEST_ELASTICITY_VERSION))
    if version > LATEST_ELASTICITY_VERSION:
        raise ElasticityConfigError(f"elasticity version {version} > supported {LATEST_ELASTICITY_VERSION}")
    prefer_larger = bool(get("prefer_larger_batch", True))
    mp = int(get("model_parallel_size", 1))
    gpn = int(get("num_gpus_per_node", 1))
    if mp > 1 and version != 0.2:
        raise ElasticityConfigError(f"elasticity v{version} does not support model parallelism (size {mp})")
    cand_micro = None
    if version == 0.2:
        if world_size == 0:
            env = os.environ.get("WORLD_SIZE", "")
            if not env.isnumeric():
                raise ElasticityConfigError("elasticity v0.2 needs the world size (argument or WORLD_SIZE)")
            world_size = int(env)
        if gpn % mp:
            raise ElasticityConfigError(f"num_gpus_per_node {gpn} must be divisible by model_parallel_size {mp}")
        dp_node = gpn // mp
        # the v0.1 search over NODES, with the batch of one data-parallel rank per node
        b_node, nodes = get_best_candidates(micro, int(max_batch / dp_node), int(min_g / gpn), int(max_g / gpn),
                                            prefer_larger)
        if nodes is None:
            raise ElasticityError(f"no valid batch size <= {max_batch} for micro batches {micro}")
        batch = int(b_node) * dp_node
        valid = [n * dp_node for n in nodes]
        if world_size // mp in valid:
            cand_micro = _largest_dividing_micro(batch, world_size, micro, prefer_larger)
        else:  # outside the set: the largest multiple of (micro x current dp size) under the cap
            dp_now = (world_size / gpn) * dp_node
            sizes = [math.floor(max_batch / float(m * dp_now)) * m * dp_now for m in micro]
            batch = int(max(sizes) if prefer_larger else min(sizes))
            valid = [int(dp_now)]
            cand_micro = _largest_dividing_micro(batch, world_size, micro, prefer_larger)
    else:
        batch, valid = get_best_candidates(micro, max_batch, min_g, max_g, prefer_larger)
        if valid is None:
            raise ElasticityError(f"no valid batch size <= {max_batch} for micro batches {micro}")
    batch = int(batch)
    if world_size > 0:
        if world_size not in valid:
            raise ElasticityIncompatibleWorldSize(f"world size {world_size} is not in the valid set {valid}")
        mb = next((m for m in sorted(micro, reverse=True) if (batch // world_size) % m == 0), None)
        if mb is None:
            raise ElasticityError(f"no micro batch divides {batch} // {world_size}")
        return batch, valid, mb
    if return_microbatch:
        if cand_micro is not None:
            return batch, valid, cand_micro
        mb = next((m for m in sorted(micro, reverse=True) if (batch // max(1, valid[0])) % m == 0), micro[0])
        return batch, valid, mb
    return batch, valid


def elasticity_enabled(ds_config):
    return bool(ds_config.get("elasticity", {}).get("enabled", False)) if isinstance(ds_config, dict) else False
