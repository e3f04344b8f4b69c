"""Runtime helpers (reference runtime/utils.py): memory reports, gradient-norm utilities,
overflow checks and uniform/balanced partitioning used by the pipeline module."""
import gc
import math

import torch

from .. import comm as dist
from ..utils.logging import logger


def see_memory_usage(message, force=False):
    """HBM allocated / peak / reserved and host RSS (reference runtime/utils.py:771). Resets the
    peak counter so consecutive calls bracket phases."""
    if not force:
        return
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    gc.collect()
    logger.info(message)
    if torch.cuda.is_available():
        g = 2 ** 30
        logger.info(f"MA {torch.cuda.memory_allocated() / g:.2f} GB  Max_MA {torch.cuda.max_memory_allocated() / g:.2f} GB  "
                    f"CA {torch.cuda.memory_reserved() / g:.2f} GB  Max_CA {torch.cuda.max_memory_reserved() / g:.2f} GB")
        torch.cuda.reset_peak_memory_stats()
    try:
        import psutil
        vm = psutil.virtual_memory()
        logger.info(f"CPU Virtual Memory: used = {(vm.total - vm.available) / 2**30:.2f} GB, percent = {vm.percent}%")
    except ImportError:
        pass


def memory_status(msg, print_rank=-1, reset_max=False):
    r = dist.get_rank() if dist.is_initialized() else 0
    if print_rank != -1 and r != print_rank:
        return
    if not torch.cuda.is_available():
        return
    g = 2 ** 30
    logger.info(f"RANK={r} MEMSTATS {msg} current alloc={torch.cuda.memory_allocated() / g:.4f}GB "
                f"(delta=n/a) max alloc={torch.cuda.max_memory_allocated() / g:.4f}GB "
                f"cache={torch.cuda.memory_reserved() / g:.4f}GB")
    if reset_max:
        torch.cuda.reset_peak_memory_stats()


def get_global_norm(norm_list):
    return math.sqrt(sum(float(n) ** 2 for n in norm_list))


def get_grad_norm(parameters, norm_type=2, mpu=None):
    """Norm of the local gradients of ``parameters`` (summed over the model-parallel group when given)."""
    ps = [p for p in parameters if p.grad is not None]
    if not ps:
        return 0.0
    if norm_type == float("inf"):
        t = torch.stack([p.grad.detach().abs().max().float() for p in ps]).max().reshape(1)
        if mpu is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=mpu.get_model_parallel_group())
        return float(t)
    t = torch.stack([p.grad.detach().float().norm(norm_type) ** norm_type for p in ps]).sum().reshape(1)
    if mpu is not None:
        dist.all_reduce(t, group=mpu.get_model_parallel_group())
    return float(t) ** (1.0 / norm_type)


def clip_grad_norm_(parameters, max_norm, norm_type=2, mpu=None):
    ps = [p for p in parameters if p.grad is not None]
    total = get_grad_norm(ps, norm_type, mpu)
    coef = max_norm / (total + 1e-6)
    if coef < 1:
        for p in ps:
            p.grad.detach().mul_(coef)
    return total


class CheckOverflow:
    """Detect inf/nan gradients across ranks (reference runtime/utils.py:CheckOverflow)."""

    def __init__(self, param_groups=None, mpu=None, zero_reduce_scatter=False, deepspeed=None):
        self.params = [p for g in (param_groups or []) for p in g]
        self.mpu = mpu

    def check(self, param_groups=None):
        ps = [p for g in param_groups for p in g] if param_groups is not None else self.params
        return self.has_overflow(ps)

    def has_overflow(self, params):
        flag = torch.zeros(1)
        for p in params:
            if p.grad is not None and not torch.isfinite(p.grad).all():
                flag.fill_(1.0)
                break
        if dist.is_initialized():
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return bool(flag.item())


def partition_uniform(num_items, num_parts):
    parts = [0] * (num_parts + 1)
    if num_items <= num_parts:
        for p in range(num_parts + 1):
            parts[p] = min(p, num_items)
        return parts
    chunk = num_items // num_parts
    rem = num_items % num_parts
    for p in range(1, num_parts + 1):
        parts[p] = parts[p - 1] + chunk + (1 if p <= rem else 0)
    return parts


def partition_balanced(weights, num_parts):
    """Contiguous parts minimising the heaviest part (binary search on the bottleneck)."""
    n = len(weights)
    pref = [0]
    for w in weights:
        pref.append(pref[-1] + w)

    def parts_for(cap):
        parts, start = [0], 0
        for _ in range(num_parts):
            end = start
            while end < n and pref[end + 1] - pref[start] <= cap:
                end += 1
            parts.append(end)
            start = end
        return parts if parts[-1] == n else None

    lo, hi = max(weights) if weights else 0, pref[-1]
    best = parts_for(hi)
    while lo < hi:
        mid = (lo + hi) // 2 if isinstance(lo, int) and isinstance(hi, int) else (lo + hi) / 2
        r = parts_for(mid)
        if r is not None:
            best, hi = r, mid
        else:
            lo = mid + (1 if isinstance(mid, int) else 1e-9)
        if not isinstance(lo, int) and hi - lo < 1e-9:
            break
    return best


def empty_cache():
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
