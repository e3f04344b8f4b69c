"""Activation checkpointing: recompute-in-backward with device RNG replay, optional partitioning of
the saved inputs across tensor-parallel ranks and optional host (pinned) offload of saved tensors.

Parity: reference runtime/activation_checkpointing/checkpointing.py -- ``CudaRNGStatesTracker``
:124, ``model_parallel_cuda_manual_seed`` :201, ``gather_partitioned_activations`` :266,
``CheckpointFunction`` :488, ``non_reentrant_checkpoint`` :704, ``checkpoint`` :948,
``configure`` :1029, ``is_configured``, ``reset``.

Design: the recompute engine is PyTorch's non-reentrant checkpoint (it composes with autograd
hooks, ZeRO-3 fetch hooks and fused weight-grad GEMMs, which the reference's reentrant Function
does not). This module adds what the reference layers on top:
  * ``partition_activations``: each TP rank keeps only 1/tp of every saved input that is identical
    across the TP group; they are all-gathered (RCCL over xGMI) just before recompute;
  * ``cpu_checkpointing``: saved inputs move to pinned host memory on a side stream and come back
    before recompute (the 288 GB HBM usually makes this unnecessary; it exists for long contexts);
  * the named device-RNG tracker so dropout inside checkpointed TP regions replays identically.
"""
import contextlib

import torch
from torch.utils.checkpoint import checkpoint as _torch_checkpoint

from ... import comm as dist
from ...accelerator import get_accelerator

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"


class _Cfg:
    configured = False
    mpu = None
    partition_activations = False
    contiguous_memory_optimization = False
    cpu_checkpointing = False
    num_checkpoints = None
    synchronize = False
    profile = False


# ------------------------------------------------------------------------------------ RNG tracker
def _device_rng_state():
    return torch.cuda.get_rng_state() if torch.cuda.is_available() else torch.get_rng_state()


def _set_device_rng_state(state):
    if torch.cuda.is_available():
        torch.cuda.set_rng_state(state)
    else:
        torch.set_rng_state(state)


class CudaRNGStatesTracker:
    """Named device RNG states; ``fork(name)`` runs a region under that state and advances it."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = dict(states)

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception(f"seed {seed} already exists")
        if name in self.states_:
            raise Exception(f"rng state {name} already exists")
        self.seeds_.add(seed)
        orig = _device_rng_state()
        if torch.cuda.is_available():
            torch.cuda.manual_seed(seed)
        else:
            torch.manual_seed(seed)
        self.states_[name] = _device_rng_state()
        _set_device_rng_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception(f"rng state {name} is not added")
        orig = _device_rng_state()
        _set_device_rng_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _device_rng_state()
            _set_device_rng_state(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    """Same default seed on every TP rank, distinct ``model-parallel-rng`` seed per TP rank."""
    from ...parallel import groups
    tp_rank = groups.get_tensor_model_parallel_rank()
    model_parallel_seed = seed + 2718 + tp_rank
    _CUDA_RNG_STATE_TRACKER.reset()
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
    else:
        torch.manual_seed(seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, model_parallel_seed)


# ------------------------------------------------------------------------------ saved-tensor hooks
def _tp_group():
    if _Cfg.mpu is not None and hasattr(_Cfg.mpu, "get_model_parallel_group"):
        return _Cfg.mpu.get_model_parallel_group()
    from ...parallel import groups
    return groups.get_tensor_model_parallel_group() if groups.get_tensor_model_parallel_world_size() > 1 else None


class _Partitioned:
    __slots__ = ("part", "shape", "numel", "group", "ws")


def _pack_partition(t):
    g = _tp_group()
    ws = dist.get_world_size(g) if g is not None else 1
    if ws <= 1 or not t.is_floating_point() or t.numel() < 1024 * ws:
        return t
    r = dist.get_rank(g)
    flat = t.detach().reshape(-1)
    n = flat.numel()
    chunk = (n + ws - 1) // ws
    padded = torch.nn.functional.pad(flat, (0, chunk * ws - n)) if chunk * ws != n else flat
    p = _Partitioned()
    p.part = padded[r * chunk:(r + 1) * chunk].clone()
    p.shape, p.numel, p.group, p.ws = t.shape, n, g, ws
    return p


def _unpack_partition(p):
    if not isinstance(p, _Partitioned):
        return p
    out = torch.empty(p.part.numel() * p.ws, dtype=p.part.dtype, device=p.part.device)
    dist.all_gather_into_tensor(out, p.part, group=p.group)
    return out[:p.numel].view(p.shape)


class _Offloaded:
    __slots__ = ("host", "device", "event")


def _pack_cpu(t):
    if not t.is_cuda or t.numel() < 4096:
        return t
    o = _Offloaded()
    o.host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    o.host.copy_(t, non_blocking=True)
    o.device = t.device
    return o


def _unpack_cpu(o):
    if not isinstance(o, _Offloaded):
        return o
    return o.host.to(o.device, non_blocking=True)


def _pack(t):
    if not torch.is_tensor(t):
        return t
    x = _pack_partition(t) if _Cfg.partition_activations else t
    if _Cfg.cpu_checkpointing:
        if isinstance(x, _Partitioned):
            x.part = _pack_cpu(x.part)
        else:
            x = _pack_cpu(x)
    return x


def _unpack(x):
    if isinstance(x, _Partitioned):
        x.part = _unpack_cpu(x.part)
        return _unpack_partition(x)
    return _unpack_cpu(x)


class CheckpointFunction(torch.autograd.Function):
    """Reentrant checkpoint whose saved inputs are partitioned across TP ranks and/or offloaded to
    pinned host memory (reference CheckpointFunction :488)."""

    @staticmethod
    def forward(ctx, run_function, n_args, *args):
        ctx.run_function = run_function
        ctx.fwd_rng = _device_rng_state()
        ctx.cpu_rng = torch.get_rng_state()
        ctx.tracker_states = get_cuda_rng_tracker().get_states()
        with torch.no_grad():
            out = run_function(*args)
        ctx.packed = [_pack(a) for a in args]
        ctx.req = [torch.is_tensor(a) and a.requires_grad for a in args]
        return out

    @staticmethod
    def backward(ctx, *grads):
        inputs = []
        for a, rg in zip(ctx.packed, ctx.req):
            t = _unpack(a)
            if torch.is_tensor(t):
                t = t.detach().requires_grad_(rg)
            inputs.append(t)
        bwd_rng, bwd_cpu = _device_rng_state(), torch.get_rng_state()
        bwd_tracker = get_cuda_rng_tracker().get_states()
        _set_device_rng_state(ctx.fwd_rng)
        torch.set_rng_state(ctx.cpu_rng)
        get_cuda_rng_tracker().set_states(ctx.tracker_states)
        with torch.enable_grad():
            out = ctx.run_function(*inputs)
        _set_device_rng_state(bwd_rng)
        torch.set_rng_state(bwd_cpu)
        get_cuda_rng_tracker().set_states(bwd_tracker)
        outs = out if isinstance(out, tuple) else (out,)
        pairs = [(o, g) for o, g in zip(outs, grads) if torch.is_tensor(o) and o.requires_grad and g is not None]
        if pairs:
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        ctx.packed = None
        return (None, None) + tuple(t.grad if torch.is_tensor(t) and t.requires_grad else None for t in inputs)


# -------------------------------------------------------------------------------------- public
def checkpoint(function, *args, **kwargs):
    """Checkpoint ``function(*args)``: only the inputs are kept; the forward is replayed in backward
    with the same device RNG state."""
    if _Cfg.synchronize and torch.cuda.is_available():
        torch.cuda.synchronize()
    if not torch.is_grad_enabled():
        return function(*args, **kwargs)
    if (_Cfg.partition_activations or _Cfg.cpu_checkpointing) and not kwargs:
        return CheckpointFunction.apply(function, len(args), *args)
    return _torch_checkpoint(function, *args, use_reentrant=False, preserve_rng_state=True, **kwargs)


def non_reentrant_checkpoint(function, *args):
    return checkpoint(function, *args)


def configure(mpu_, deepspeed_config=None, partition_activations=None, contiguous_checkpointing=None,
              num_checkpoints=None, checkpoint_in_cpu=None, synchronize=None, profile=None):
    """Set the policy from the engine config block ``activation_checkpointing`` and/or kwargs."""
    _Cfg.mpu = mpu_
    if deepspeed_config is not None:
        ac = deepspeed_config.model.activation_checkpointing if hasattr(deepspeed_config, "model") else \
            deepspeed_config
        _Cfg.partition_activations = ac.partition_activations
        _Cfg.contiguous_memory_optimization = ac.contiguous_memory_optimization
        _Cfg.cpu_checkpointing = ac.cpu_checkpointing
        _Cfg.num_checkpoints = ac.number_checkpoints
        _Cfg.synchronize = ac.synchronize_checkpoint_boundary
        _Cfg.profile = ac.profile
    for k, v in dict(partition_activations=partition_activations, contiguous_memory_optimization=contiguous_checkpointing,
                     num_checkpoints=num_checkpoints, cpu_checkpointing=checkpoint_in_cpu, synchronize=synchronize,
                     profile=profile).items():
        if v is not None:
            setattr(_Cfg, k, v)
    if _Cfg.cpu_checkpointing and not get_accelerator().gpu:
        _Cfg.cpu_checkpointing = False  # already on the host
    _Cfg.configured = True


def is_configured():
    return _Cfg.configured


def reset():
    """Reset per-iteration state (kept for API parity; nothing is buffered between iterations)."""
    return None


def set_num_layers(nlayers):
    _Cfg.num_checkpoints = nlayers
