"""``zero.Init`` and ``GatheredParameters`` (parity: reference runtime/zero/partition_parameters.py:879
``Init``, :1141 ``_post_init_method``, :1109-1116 ``_zero_init_param`` broadcast, :2193
``GatheredParameters``).

Partition at construction. Inside ``with zero.Init():`` every ``nn.Module`` subclass constructor is
wrapped; when a module's OUTERMOST constructor returns, each of its parameters that is still whole is

  1. broadcast from the group's first rank (so every rank starts from identical weights whatever
     its RNG state -- no full-model broadcast later in the engine), and
  2. cut to this rank's 1/W chunk of the flattened tensor (``p.ds_tensor``; ``p.data`` becomes an
     empty tensor that keeps dtype/device).

Children finish before their parents, so at any moment at most ONE module's own parameters exist
in full: peak memory during construction is (full model / W) + (largest module's own params). For
Llama-3-70B (141 GB bf16) on 8 MI355X that is 17.6 GB + one decoder layer (1.7 GB) per GPU instead
of 141 GB. ZeRO-3 then regroups the per-parameter chunks into its flat units (``stage3._make_unit``,
one unit gathered at a time) and frees the construction partitions.

Initialising partitioned weights: an element-wise i.i.d. init (``normal_``, ``uniform_``, ``zero_``)
applied to a partition is distributed exactly like the same init on the full tensor, so model code
can initialise ``zero.local_shard(p)`` instead of ``p`` (models/llama.py does); inits that need the
whole tensor (orthogonal, copies from another module) run under ``GatheredParameters(...,
modifier_rank=0)`` before ``initialize()``, as with the reference.

``partition=None`` (default) partitions whenever the group has more than one rank; at W = 1 the
model is built whole (ZeRO-3 keeps every unit resident there anyway). With 288 GB of HBM per
GPU the whole of an 8B model fits on every rank, but a 70B model does not fit next to its
optimizer state without this.
"""
import contextlib
import functools

import torch
import torch.nn as nn

from ... import comm as dist
from ...accelerator import get_accelerator

_ACTIVE = []  # stack of active Init contexts (nesting is allowed; the innermost one partitions)


def _all_module_classes():
    seen, stack = set(), [nn.Module]
    while stack:
        c = stack.pop()
        for s in c.__subclasses__():
            if s not in seen:
                seen.add(s)
                stack.append(s)
    return seen


def _wrap_ctor(cls):
    orig = cls.__dict__.get("__init__")
    if orig is None or getattr(orig, "_sxe_zero_init_orig", None) is not None:
        return None

    @functools.wraps(orig)
    def ctor(mod, *args, **kwargs):
        d = mod.__dict__
        d["_sxe_ctor_depth"] = d.get("_sxe_ctor_depth", 0) + 1
        try:
            orig(mod, *args, **kwargs)
        finally:
            d["_sxe_ctor_depth"] -= 1
        if d["_sxe_ctor_depth"] == 0:
            del d["_sxe_ctor_depth"]
            if _ACTIVE:
                _ACTIVE[-1]._post_init(mod)

    ctor._sxe_zero_init_orig = orig
    cls.__init__ = ctor
    return orig


class Init:
    """Construct modules directly on the GPU in the training dtype, partitioned over
    ``data_parallel_group`` (see the module docstring).

    ``remote_device="cpu"`` keeps the construction partitions in (pinned) host memory.
    ``stats`` reports what construction held: ``peak_full_numel`` (largest number of elements that
    existed unpartitioned at once), ``partition_numel`` (elements of this rank's partitions) and
    ``params`` (parameters partitioned)."""

    def __init__(self, module=None, data_parallel_group=None, mem_efficient_linear=True, remote_device=None,
                 pin_memory=False, config_dict_or_path=None, config=None, enabled=True, dtype=None, mpu=None,
                 zero_param_parallel_group=None, zero_quantized_weights=False, zero_quantized_nontrainable_weights=False,
                 sequence_data_parallel_group=None, param_swapper=None, partition=None):
        self.enabled = enabled
        self.dtype = dtype or torch.bfloat16
        acc = get_accelerator()
        if not dist.is_initialized() and enabled:
            dist.init_distributed(verbose=False)
        self.compute_device = torch.device(acc.current_device_name())
        self.host = remote_device in ("cpu", "nvme")
        self.device = torch.device("cpu") if self.host else self.compute_device
        self.pin_memory = bool(pin_memory) and self.device.type == "cpu" and acc.gpu
        self.group = data_parallel_group if data_parallel_group is not None else sequence_data_parallel_group
        W = dist.get_world_size(self.group)
        self.partition = (W > 1) if partition is None else bool(partition)
        self.world = W
        self.rank = dist.get_rank(self.group)
        self.src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
        self.stats = {"peak_full_numel": 0, "partition_numel": 0, "params": 0}
        self._wrapped = {}
        if module is not None and enabled:
            module.to(device=self.device, dtype=self.dtype)
            if self.partition:
                for m in module.modules():
                    self._partition_own(m, recurse=False)

    def __enter__(self):
        if not self.enabled:
            return self
        self._prev_dtype = torch.get_default_dtype()
        torch.set_default_dtype(self.dtype)
        self._dev_ctx = torch.device(self.device)
        self._dev_ctx.__enter__()
        if self.partition:
            for cls in _all_module_classes():
                orig = _wrap_ctor(cls)
                if orig is not None:
                    self._wrapped[cls] = orig
            # classes defined while the context is open get wrapped too
            self._prev_init_subclass = nn.Module.__dict__.get("__init_subclass__")
            wrapped = self._wrapped

            def init_subclass(cls, **kw):
                orig = _wrap_ctor(cls)
                if orig is not None:
                    wrapped[cls] = orig
            nn.Module.__init_subclass__ = classmethod(init_subclass)
        _ACTIVE.append(self)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        _ACTIVE.remove(self)
        self._dev_ctx.__exit__(*exc)
        torch.set_default_dtype(self._prev_dtype)
        if self.partition:
            if self._prev_init_subclass is not None:
                nn.Module.__init_subclass__ = self._prev_init_subclass
            else:
                del nn.Module.__init_subclass__
            if not _ACTIVE:  # restore the original constructors (an outer Init keeps its wraps)
                for cls, orig in self._wrapped.items():
                    cls.__init__ = orig
            self._wrapped = {}
        return False

    # --------------------------------------------------------------------------------------------
    def _post_init(self, mod):
        if not self.partition:
            return
        whole = [p for p in mod.parameters() if not hasattr(p, "ds_tensor") and not hasattr(p, "_sxe_init_local")]
        n = sum(p.numel() for p in whole)
        self.stats["peak_full_numel"] = max(self.stats["peak_full_numel"], n)
        for p in whole:
            if getattr(p, "allreduce", True) is False:
                # expert-parallel weights differ across the expert-parallel group (reference
                # moe/experts.py marks them allreduce=False): they keep their local init, unpartitioned
                p._sxe_init_local = True
                continue
            self._partition_param(p)

    def _partition_own(self, mod, recurse=False):
        for p in mod.parameters(recurse=recurse):
            if not hasattr(p, "ds_tensor") and getattr(p, "allreduce", True) is not False:
                self._partition_param(p)

    def _partition_param(self, p):
        if p.dtype.is_floating_point and p.dtype != self.dtype:
            p.data = p.data.to(self.dtype)
        if self.world > 1:
            comm_t = p.data if p.data.device.type == self.compute_device.type or dist.get_backend() == "gloo" \
                else p.data.to(self.compute_device)
            dist.broadcast(comm_t, src=self.src, group=self.group)
            if comm_t is not p.data:
                p.data.copy_(comm_t)
        _partition_param(p, self.group, pin=self.pin_memory)
        self.stats["partition_numel"] += p.ds_tensor.numel()
        self.stats["params"] += 1


def _partition_param(p, group=None, pin=False):
    """Keep this rank's 1/W chunk of the flattened parameter as ``p.ds_tensor``."""
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    n = p.numel()
    chunk = (n + W - 1) // W
    flat = p.data.reshape(-1)
    lo, hi = min(n, r * chunk), min(n, (r + 1) * chunk)
    shard = torch.zeros(chunk, dtype=p.dtype, device=p.device, pin_memory=pin)
    shard[:hi - lo].copy_(flat[lo:hi])
    p.ds_tensor = shard
    p.ds_shape = p.shape
    p.ds_numel = n
    p.ds_group = group
    p.ds_valid = hi - lo  # elements of the shard that belong to the parameter (the rest is padding)
    p.ds_tensor_full = functools.partial(_gather_full, p)
    p.data = torch.empty(0, dtype=p.dtype, device=p.device)


def _gather_full(p, device=None):
    """All-gather the construction partitions of ``p`` into a new full tensor."""
    group, shard = p.ds_group, p.ds_tensor
    W = dist.get_world_size(group)
    dev = device or shard.device
    if dist.get_backend() == "nccl":
        dev = torch.device(get_accelerator().current_device_name())
    src = shard.to(dev, non_blocking=True)
    out = torch.empty(shard.numel() * W, dtype=shard.dtype, device=dev)
    if W > 1:
        dist.all_gather_into_tensor(out, src, group=group)
    else:
        out.copy_(src)
    return out[:p.ds_numel].view(p.ds_shape)


def release_construction_partition(p):
    """Drop the ``zero.Init`` partition of ``p`` once ZeRO-3 owns the parameter's data."""
    for a in ("ds_tensor", "ds_tensor_full", "ds_valid"):
        if hasattr(p, a):
            delattr(p, a)


def local_shard(p):
    """The part of this rank's construction partition that belongs to ``p`` (``p`` itself when it
    is not partitioned). Element-wise initialisers applied to it initialise ``p`` in distribution."""
    if hasattr(p, "ds_tensor"):
        return p.ds_tensor[:p.ds_valid]
    return p


def is_zero_param(p):
    return hasattr(p, "ds_tensor") or hasattr(p, "ds_unit")


class GatheredParameters:
    """Temporarily materialise ZeRO-3 partitioned parameters. With ``modifier_rank`` set, edits made
    on that rank are broadcast and written back into the partitions (and fp32 masters) on exit.

    Works both for parameters owned by a ZeRO-3 engine (``ds_unit``) and for parameters still in
    their ``zero.Init`` construction partitions (``ds_tensor``), e.g. for a whole-tensor init
    between construction and ``initialize()``."""

    def __init__(self, params, modifier_rank=None, fwd_module=None, enabled=True):
        if isinstance(params, torch.nn.Parameter) or isinstance(params, torch.Tensor):
            params = [params]
        params = list(params)
        self.params = [p for p in params if hasattr(p, "ds_unit")]
        self.init_params = [p for p in params if hasattr(p, "ds_tensor") and not hasattr(p, "ds_unit")]
        self.modifier_rank = modifier_rank
        self.enabled = enabled and bool(self.params or self.init_params)
        self.units = []

    def __enter__(self):
        if not self.enabled:
            return self
        for p in self.init_params:
            p.data = _gather_full(p, device=p.ds_tensor.device).to(p.ds_tensor.device)
        if self.params:
            owner = self.params[0].ds_unit.owner
            self.owner = owner
            self.units = owner.gather_params(self.params)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        for p in self.init_params:
            if self.modifier_rank is not None and dist.get_world_size(p.ds_group) > 1:
                src = dist.get_global_rank(p.ds_group, self.modifier_rank) if p.ds_group is not None \
                    else self.modifier_rank
                t = p.data
                if dist.get_backend() == "nccl" and t.device.type == "cpu":
                    t = t.to(get_accelerator().current_device_name())
                dist.broadcast(t, src=src, group=p.ds_group)
                if t is not p.data:
                    p.data.copy_(t)
            W, r = dist.get_world_size(p.ds_group), dist.get_rank(p.ds_group)
            chunk = p.ds_tensor.numel()
            lo = min(p.ds_numel, r * chunk)
            p.ds_tensor[:p.ds_valid].copy_(p.data.reshape(-1)[lo:lo + p.ds_valid])
            p.data = torch.empty(0, dtype=p.dtype, device=p.ds_tensor.device)
        if self.units:
            if self.modifier_rank is not None:
                group = self.owner.topo.slice_group
                src = self.owner.topo.slice_ranks[self.modifier_rank] if self.owner.topo.slice_ranks else self.modifier_rank
                self.owner.commit_modified_units(self.units, src_rank=src if dist.get_world_size() > 1 else None,
                                                 group=group)
            for u in self.units:
                self.owner._release_unit(u)
        return False


@contextlib.contextmanager
def gather_all(engine_or_optimizer):
    opt = getattr(engine_or_optimizer, "optimizer", engine_or_optimizer)
    opt.gather_all()
    try:
        yield
    finally:
        opt.release_all()


def register_external_parameter(module, parameter):
    """Declare that ``module``'s forward uses ``parameter`` although another module owns it
    (reference partition_parameters.py ``register_external_parameter``): under ZeRO-3 the module's
    fetch then gathers the owning unit as well. Call before ``initialize()``. Parameters of a
    module that are owned by another unit (tied weights) are detected automatically."""
    lst = getattr(module, "_sxe_external_params", None)
    if lst is None:
        lst = []
        module._sxe_external_params = lst
    if all(p is not parameter for p in lst):
        lst.append(parameter)


def unregister_external_parameter(module, parameter):
    lst = getattr(module, "_sxe_external_params", [])
    module._sxe_external_params = [p for p in lst if p is not parameter]
