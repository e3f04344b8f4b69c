"""Full / local views of ZeRO-partitioned fp32 parameters, gradients and optimizer state.

Parity: reference utils/tensor_fragment.py (``safe_get_full_fp32_param`` / ``safe_get_full_grad`` /
``safe_get_full_optimizer_state`` / ``safe_set_full_fp32_param`` / ``safe_set_full_optimizer_state``
and the ``safe_*_local_*`` variants, built on the lp->hp linkage of
utils/mixed_precision_linkage.py:11-51). Here every ZeRO stage (0/1/2/3, with or without
Shuffle-exchange slices, with ZeRO-Offload) shares one layout -- flat units split into S equal
chunks (runtime/zero/flat.py) -- so a parameter's fragment on this rank is just the intersection of
its [offset, offset+numel) range with the rank's chunk, and the full tensor is ONE all-reduce of
the zero-padded fragments over the partition group. Call these between ``backward`` and ``step``
for gradients (the accumulator is cleared after the step), at any time for parameters / state.
All ranks of the partition group must call the ``full`` getters together (collective).
"""
import torch

from .. import comm as dist


def _loc(param):
    loc = getattr(param, "_sxe_zero", None)
    if loc is None:
        raise ValueError("parameter is not managed by a ZeRO optimizer of this framework")
    if hasattr(loc[0], "wait_params"):  # overlapped optimizer updates still in flight
        loc[0].wait_params()
    return loc  # (optimizer, group index, unit, param index in unit)


def _fragment(param, which, key=None):
    """(fragment tensor of this rank's chunk, (param_lo, param_hi)) or (None, None)."""
    opt, g, u, i = _loc(param)
    if which == "grad" and hasattr(opt, "_zero_stale"):
        opt._zero_stale()  # ZeRO-3 zeroes accumulator slots lazily: settle them before reading
    rng = u.param_range_in_shard(i)
    if rng is None:
        return None, None
    plo, phi, slo = rng
    n = phi - plo
    if which == "param":
        src = u.master
        if src is None:  # NVMe-offloaded masters: the bit16 shard is the freshest device copy
            return u.shard[slo:slo + n].float(), (plo, phi)
        return src[slo:slo + n], (plo, phi)
    if which == "grad":
        return u.grad[slo:slo + n], (plo, phi)
    st = opt.optimizer.state[opt.master[g]]
    if key not in st:
        raise KeyError(f"optimizer state has no {key!r} (have {list(st)})")
    flat = st[key]
    base = opt._unit_offsets(g)[opt.units[g].index(u)]
    return flat[base + slo:base + slo + n], (plo, phi)


def _full(param, which, key=None):
    opt, g, u, i = _loc(param)
    frag, rng = _fragment(param, which, key)
    full = torch.zeros(u.numels[i], dtype=torch.float32, device=u.grad.device)
    if frag is not None:
        full[rng[0]:rng[1]].copy_(frag.reshape(-1).to(full.device, torch.float32))
    grp = opt.partition_group
    if u.S > 1 and grp is not None:
        dist.all_reduce(full, group=grp)
    return full.view(u.shapes[i])


def safe_get_full_fp32_param(param):
    return _full(param, "param")


def safe_get_full_grad(param):
    return _full(param, "grad")


def safe_get_full_optimizer_state(param, optim_state_key):
    return _full(param, "state", optim_state_key)


def safe_get_local_fp32_param(param):
    """This rank's fragment (flattened), or an empty tensor when the rank holds none of it."""
    frag, _ = _fragment(param, "param")
    return frag if frag is not None else torch.empty(0)


def safe_get_local_grad(param):
    frag, _ = _fragment(param, "grad")
    return frag if frag is not None else torch.empty(0)


def safe_get_local_optimizer_state(param, optim_state_key):
    frag, _ = _fragment(param, "state", optim_state_key)
    return frag if frag is not None else torch.empty(0)


@torch.no_grad()
def safe_set_full_fp32_param(param, value):
    """Overwrite the fp32 master (and the bit16 working copy) of ``param`` with the full ``value``
    (identical on every rank of the partition group)."""
    opt, g, u, i = _loc(param)
    v = value.reshape(-1).to(torch.float32)
    rng = u.param_range_in_shard(i)
    if rng is not None:
        plo, phi, slo = rng
        if u.master is not None:
            u.master[slo:slo + phi - plo].copy_(v[plo:phi].to(u.master.device))
        u.shard[slo:slo + phi - plo].copy_(v[plo:phi].to(u.shard.device, u.shard.dtype))
    if u.flat is not None and u.flat.untyped_storage().size() > 0:
        o, n = u.offsets[i], u.numels[i]
        u.flat[o:o + n].copy_(v.to(u.flat.device, u.flat.dtype))
    _weights_rewritten()


def _weights_rewritten():
    """The bit16 weights changed outside the optimizer step: drop cached transposes (ops/linear.py)."""
    from ..ops.linear import invalidate_transposed_weights
    invalidate_transposed_weights()


@torch.no_grad()
def safe_set_full_optimizer_state(param, value, optim_state_key):
    frag, rng = _fragment(param, "state", optim_state_key)
    if frag is not None:
        frag.copy_(value.reshape(-1)[rng[0]:rng[1]].to(frag.device, frag.dtype))


@torch.no_grad()
def safe_set_full_grad(param, value):
    frag, rng = _fragment(param, "grad")
    if frag is not None:
        frag.copy_(value.reshape(-1)[rng[0]:rng[1]].to(frag.device, frag.dtype))


@torch.no_grad()
def safe_set_local_fp32_param(param, value):
    opt, g, u, i = _loc(param)
    rng = u.param_range_in_shard(i)
    if rng is None:
        return
    plo, phi, slo = rng
    if u.master is not None:
        u.master[slo:slo + phi - plo].copy_(value.reshape(-1).to(u.master.device))
    u.shard[slo:slo + phi - plo].copy_(value.reshape(-1).to(u.shard.device, u.shard.dtype))
    _weights_rewritten()


@torch.no_grad()
def safe_set_local_optimizer_state(param, value, optim_state_key):
    frag, _ = _fragment(param, "state", optim_state_key)
    if frag is not None:
        frag.copy_(value.reshape(-1).to(frag.device, frag.dtype))


@torch.no_grad()
def safe_set_local_grad(param, value):
    frag, _ = _fragment(param, "grad")
    if frag is not None:
        frag.copy_(value.reshape(-1).to(frag.device, frag.dtype))
