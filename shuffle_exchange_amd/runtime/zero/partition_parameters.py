"""``zero.Init`` and ``GatheredParameters`` (parity: reference runtime/zero/partition_parameters.py:879
``Init``, :2193 ``GatheredParameters``).

MI355X sizing note: with 288 GB of HBM per GPU a 70B-parameter model fits *unpartitioned* in bf16
(140 GB) on every GPU, so ``Init`` constructs modules directly on the GPU in the training dtype
(no fp32 host materialisation: ``remote_device``/``dtype`` honoured) and ZeRO-3 partitions them
unit by unit when the engine is built (peak = full model + one unit). With ``partition=True``
each module is additionally partitioned right after its constructor returns (per-parameter
``ds_tensor`` chunks, gathered again one unit at a time by the engine) for models that do not fit.
"""
import contextlib

import torch

from ... import comm as dist
from ...accelerator import get_accelerator


class Init:
    def __init__(self, module=None, data_parallel_group=None, mem_efficient_linear=True, remote_device=None,
                 pin_memory=False, config_dict_or_path=None, config=None, enabled=True, dtype=None, mpu=None,
                 zero_param_parallel_group=None, zero_quantized_weights=False, zero_quantized_nontrainable_weights=False,
                 sequence_data_parallel_group=None, param_swapper=None, partition=False):
        self.enabled = enabled
        self.dtype = dtype or torch.bfloat16
        acc = get_accelerator()
        if remote_device in (None, "none", "device", "cuda"):
            self.device = torch.device(acc.current_device_name())
        else:
            self.device = torch.device("cpu")
        self.partition = partition
        self.group = data_parallel_group
        self._prev = None
        self._orig_init = None
        self._created = []
        if module is not None and enabled:
            module.to(device=self.device, dtype=self.dtype)

    def __enter__(self):
        if not self.enabled:
            return self
        self._prev_dtype = torch.get_default_dtype()
        torch.set_default_dtype(self.dtype)
        self._dev_ctx = torch.device(self.device)
        self._dev_ctx.__enter__()
        if self.partition:
            orig = torch.nn.Module.__init__
            outer = self

            def patched(mod, *a, **k):
                orig(mod, *a, **k)
                outer._created.append(mod)
            self._orig_init = orig
            torch.nn.Module.__init__ = patched
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        self._dev_ctx.__exit__(*exc)
        torch.set_default_dtype(self._prev_dtype)
        if self.partition:
            torch.nn.Module.__init__ = self._orig_init
            seen = set()
            for m in self._created:
                for p in m.parameters(recurse=False):
                    if id(p) not in seen:
                        seen.add(id(p))
                        _partition_param(p, self.group)
        return False


def _partition_param(p, group=None):
    """Keep this rank's 1/W chunk of the flattened parameter as ``p.ds_tensor``."""
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    n = p.numel()
    chunk = (n + W - 1) // W
    flat = torch.zeros(chunk * W, dtype=p.dtype, device=p.device)
    flat[:n].copy_(p.data.reshape(-1))
    p.ds_tensor = flat[r * chunk:(r + 1) * chunk].clone()
    p.ds_shape = p.shape
    p.ds_numel = n
    p.ds_group = group

    def full():
        out = torch.empty(chunk * W, dtype=p.ds_tensor.dtype, device=p.ds_tensor.device)
        dist.all_gather_into_tensor(out, p.ds_tensor, group=group)
        return out[:n].view(p.ds_shape)
    p.ds_tensor_full = full
    p.data = torch.empty(0, dtype=p.dtype, device=p.device)


class GatheredParameters:
    """Temporarily materialise ZeRO-3 partitioned parameters. With ``modifier_rank`` set, edits made
    on that rank are broadcast and written back into the partitions (and fp32 masters) on exit."""

    def __init__(self, params, modifier_rank=None, fwd_module=None, enabled=True):
        if isinstance(params, torch.nn.Parameter) or isinstance(params, torch.Tensor):
            params = [params]
        self.params = [p for p in params if hasattr(p, "ds_unit")]
        self.modifier_rank = modifier_rank
        self.enabled = enabled and bool(self.params)
        self.units = []

    def __enter__(self):
        if not self.enabled:
            return self
        owner = self.params[0].ds_unit.owner
        self.owner = owner
        self.units = owner.gather_params(self.params)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
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
