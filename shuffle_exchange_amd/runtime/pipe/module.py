"""Pipeline-parallel model description: ``LayerSpec`` / ``TiedLayerSpec`` lists partitioned over
pipeline stages.

Parity: reference runtime/pipe/module.py -- ``LayerSpec`` :25, ``TiedLayerSpec`` :70,
``PipelineModule`` :86 (partitioning ``_partition_layers`` :393 with methods ``uniform`` /
``parameters`` / ``type:<regex>``, tied modules ``_index_tied_modules`` :454 and
``allreduce_tied_weight_gradients``, activation-checkpoint intervals, layer-wise checkpoint files
``layer_XX-model_states.pt``).

Differences by design: parameter counts for the ``parameters`` method are taken from a build on the
``meta`` device (no host memory, no init cost) and the partition is the exact min-max contiguous
split (binary search over the bottleneck), not a heuristic.
"""
import os
import re
from functools import partial

import torch
import torch.nn as nn

from ... import comm as dist
from ...parallel.topology import PipeDataParallelTopology, PipelineParallelGrid, ProcessTopology
from ...utils.logging import log_dist


class LayerSpec:
    """Delays construction of a layer until the stage that owns it builds it."""

    def __init__(self, typename, *module_args, **module_kwargs):
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs
        if not issubclass(typename, nn.Module):
            raise RuntimeError("LayerSpec only supports torch.nn.Module types")

    def __repr__(self):
        return f"LayerSpec({self.typename.__name__})"

    def build(self, log=False):
        if log:
            log_dist(f"building {self!r}", ranks=[0])
        return self.typename(*self.module_args, **self.module_kwargs)


class TiedLayerSpec(LayerSpec):
    """A layer whose ``tied_weight_attr`` parameters are shared by every stage holding ``key``."""

    def __init__(self, key, typename, *module_args, forward_fn=None, tied_weight_attr=("weight",),
                 **module_kwargs):
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = [tied_weight_attr] if isinstance(tied_weight_attr, str) else list(tied_weight_attr)


def partition_uniform(num_items, num_parts):
    """Boundaries (num_parts + 1) splitting num_items as evenly as possible."""
    base, extra = divmod(num_items, num_parts)
    parts = [0]
    for p in range(num_parts):
        parts.append(parts[-1] + base + (1 if p < extra else 0))
    return parts


def partition_balanced(weights, num_parts):
    """Contiguous split of ``weights`` into ``num_parts`` minimising the largest part."""
    n = len(weights)
    if num_parts >= n:
        return partition_uniform(n, num_parts)
    prefix = [0]
    for w in weights:
        prefix.append(prefix[-1] + w)

    def cuts_for(limit):
        parts, start = [0], 0
        for _ in range(num_parts):
            end = start
            while end < n and prefix[end + 1] - prefix[start] <= limit:
                end += 1
            if end == start and start < n:
                return None  # a single item exceeds the limit
            parts.append(end)
            start = end
        return parts if parts[-1] == n else None

    lo, hi = max(weights), prefix[-1]
    while lo < hi:
        mid = (lo + hi) // 2
        if cuts_for(mid) is not None:
            hi = mid
        else:
            lo = mid + 1
    parts = cuts_for(lo)
    # give empty trailing stages at least nothing-breaking boundaries (monotone by construction)
    return parts


class PipelineModule(nn.Module):
    is_pipeline_module = True

    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seed_layers=False, seed_fn=None,
                 base_seed=1234, partition_method="parameters", activation_checkpoint_interval=0,
                 activation_checkpoint_func=None, checkpointable_layers=None):
        super().__init__()
        if num_stages is None and topology is None:
            raise RuntimeError("must provide num_stages or topology")
        dist.init_distributed()
        self.world_size = dist.get_world_size()
        self.global_rank = dist.get_rank()
        if topology is None:
            assert self.world_size % num_stages == 0, "world size must be divisible by num_stages"
            topology = PipeDataParallelTopology(num_pp=num_stages, num_dp=self.world_size // num_stages)
        self._topo = topology
        self.num_stages = topology.get_dim("pipe")
        self._grid = PipelineParallelGrid(topology=topology)
        self.stage_id = self._grid.get_stage_id()
        self.loss_fn = loss_fn
        self.seed_layers, self.seed_fn, self.base_seed = seed_layers, seed_fn, base_seed
        self.activation_checkpoint_interval = int(activation_checkpoint_interval or 0)
        self.activation_checkpoint_func = activation_checkpoint_func
        self.checkpointable_layers = checkpointable_layers
        self._layer_specs = list(layers)
        self._num_layers = len(self._layer_specs)
        self.partition_method = partition_method
        self.parts = self._partition_layers(partition_method)
        self._local_start = self.parts[self.stage_id]
        self._local_stop = self.parts[self.stage_id + 1]
        self.tied_modules = nn.ModuleDict()
        self.tied_weight_attrs = {}
        self.forward_funcs = []
        self._build()
        self.tied_comms = self._index_tied_modules()
        self._synchronize_tied_weights()

    # ----------------------------------------------------------------------------- partitioning
    def _layer_weight(self, spec):
        if isinstance(spec, LayerSpec):
            with torch.device("meta"):
                m = spec.build()
            return sum(p.numel() for p in m.parameters() if p.requires_grad)
        if isinstance(spec, nn.Module):
            return sum(p.numel() for p in spec.parameters() if p.requires_grad)
        return 0

    def _layer_name(self, spec):
        if isinstance(spec, LayerSpec):
            return spec.typename.__name__
        if isinstance(spec, nn.Module):
            return spec.__class__.__name__
        return getattr(spec, "__name__", type(spec).__name__)

    def _partition_layers(self, method):
        S, n = self.num_stages, self._num_layers
        m = method.lower()
        if m == "uniform":
            parts = partition_uniform(n, S)
        elif m == "parameters":
            parts = partition_balanced([self._layer_weight(s) for s in self._layer_specs], S)
        elif m.startswith("type:"):
            pat = method.split(":", 1)[1]
            weights = [1 if re.search(pat, self._layer_name(s), re.IGNORECASE) else 0 for s in self._layer_specs]
            if sum(weights) == 0:
                parts = partition_uniform(n, S)
            else:
                # balance the matching layers; non-matching ones ride along with their neighbours
                idx = [i for i, w in enumerate(weights) if w]
                cuts = partition_uniform(len(idx), S)
                parts = [0] + [idx[c] if c < len(idx) else n for c in cuts[1:-1]] + [n]
        elif m == "profile":
            raise NotImplementedError("partition_method='profile' is not implemented (the reference does not either)")
        else:
            raise NotImplementedError(f"partition method {method}")
        if self.global_rank == 0:
            for s in range(S):
                names = [self._layer_name(x) for x in self._layer_specs[parts[s]:parts[s + 1]]]
                log_dist(f"pipeline stage {s}: layers [{parts[s]}, {parts[s + 1]}) {names}", ranks=[0])
        return parts

    # ----------------------------------------------------------------------------------- build
    def _build(self):
        for local_i, spec in enumerate(self._layer_specs[self._local_start:self._local_stop]):
            idx = self._local_start + local_i
            if self.seed_layers:
                (self.seed_fn or torch.manual_seed)(self.base_seed + idx)
            if isinstance(spec, TiedLayerSpec):
                if spec.key not in self.tied_modules:
                    self.tied_modules[spec.key] = spec.build()
                    self.tied_weight_attrs[spec.key] = spec.tied_weight_attr
                mod = self.tied_modules[spec.key]
                self.forward_funcs.append(partial(spec.forward_fn, mod) if spec.forward_fn is not None else mod)
            elif isinstance(spec, LayerSpec):
                mod = spec.build()
                self.add_module(str(idx), mod)
                self.forward_funcs.append(mod)
            elif isinstance(spec, nn.Module):
                self.add_module(str(idx), spec)
                self.forward_funcs.append(spec)
            else:
                self.forward_funcs.append(spec)  # plain callable (e.g. a lambda reshaping the activation)

    # ----------------------------------------------------------------------------------- tied
    def _index_tied_modules(self):
        """One process group per (tied key, data/model coordinate) over the stages holding the key."""
        comms = {}
        keys_by_stage = []
        for s in range(self.num_stages):
            ks = set()
            for spec in self._layer_specs[self.parts[s]:self.parts[s + 1]]:
                if isinstance(spec, TiedLayerSpec):
                    ks.add(spec.key)
            keys_by_stage.append(ks)
        all_keys = sorted(set().union(*keys_by_stage)) if keys_by_stage else []
        other_axes = [a for a in self._topo.get_axis_names() if a != "pipe"]
        import itertools
        for key in all_keys:
            stages = [s for s in range(self.num_stages) if key in keys_by_stage[s]]
            if len(stages) < 2:
                continue
            for coord in itertools.product(*[range(self._topo.get_dim(a)) for a in other_axes]):
                kw = dict(zip(other_axes, coord))
                ranks = sorted(self._topo.get_rank(pipe=s, **kw) for s in stages)
                g = dist.new_group(ranks)
                if self.global_rank in ranks:
                    mod = self.tied_modules[key]
                    comms[key] = {"ranks": ranks, "group": g, "module": mod,
                                  "weight_attr": self.tied_weight_attrs[key]}
        return comms

    def _tied_params(self, key):
        c = self.tied_comms[key]
        return [getattr(c["module"], a) for a in c["weight_attr"]]

    def _synchronize_tied_weights(self):
        for key, c in self.tied_comms.items():
            for p in self._tied_params(key):
                dist.broadcast(p.data, src=min(c["ranks"]), group=c["group"])

    def allreduce_tied_weight_gradients(self):
        for key, c in self.tied_comms.items():
            for p in self._tied_params(key):
                if p.grad is not None:
                    dist.all_reduce(p.grad, group=c["group"])

    def get_tied_weights_and_groups(self):
        return [(p, c["group"]) for key, c in self.tied_comms.items() for p in self._tied_params(key)]

    def tied_parameters(self):
        return [p for key in self.tied_comms for p in self._tied_params(key)]

    # --------------------------------------------------------------------------------- forward
    def forward(self, forward_input):
        def run(start, end):
            def fn(*inputs):
                x = inputs[0] if len(inputs) == 1 else inputs
                for f in self.forward_funcs[start:end]:
                    x = f(x)
                return x
            return fn

        n = len(self.forward_funcs)
        if self.activation_checkpoint_interval <= 0 or not (self.training and torch.is_grad_enabled()):
            return run(0, n)(forward_input)
        from torch.utils.checkpoint import checkpoint
        ck = self.activation_checkpoint_func or (lambda f, *a: checkpoint(f, *a, use_reentrant=False))
        x = forward_input
        for s in range(0, n, self.activation_checkpoint_interval):
            e = min(s + self.activation_checkpoint_interval, n)
            args = x if isinstance(x, tuple) else (x,)
            if self._is_checkpointable(self.forward_funcs[s:e]):
                x = ck(run(s, e), *args)
            else:
                x = run(s, e)(*args)
        return x

    def _is_checkpointable(self, funcs):
        if self.checkpointable_layers is not None:
            return all(f.__class__.__name__ in self.checkpointable_layers for f in funcs)
        return any(isinstance(f, nn.Module) and any(True for _ in f.parameters()) for f in funcs)

    # ----------------------------------------------------------------------------- accessors
    def topology(self):
        return self._topo

    def mpu(self):
        return self._grid

    def num_pipeline_stages(self):
        return self.num_stages

    def stage_owner(self, layer_idx):
        for s in range(self.num_stages):
            if self.parts[s] <= layer_idx < self.parts[s + 1]:
                return s
        raise RuntimeError(f"layer {layer_idx} out of range")

    # ------------------------------------------------------------------------- checkpointing
    def ckpt_layer_path(self, ckpt_dir, local_layer_idx):
        idx = self._local_start + local_layer_idx
        rank_repr = self._grid._topo.get_rank_repr(rank=self.global_rank)
        suffix = f"-{rank_repr}" if rank_repr else ""
        return os.path.join(ckpt_dir, f"layer_{idx:02d}{suffix}-model_states.pt")

    def save_state_dict(self, save_dir, checkpoint_engine=None, exclude_frozen_params=False):
        """Each layer to its own file; data-parallel rank 0 of each stage writes."""
        if self._grid.data_parallel_id != 0:
            return
        os.makedirs(save_dir, exist_ok=True)
        for i, f in enumerate(self.forward_funcs):
            if not isinstance(f, nn.Module) or not list(f.state_dict().keys()):
                continue
            sd = {k: v.detach().clone() for k, v in f.state_dict().items()}
            if exclude_frozen_params:
                frozen = {n for n, p in f.named_parameters() if not p.requires_grad}
                sd = {k: v for k, v in sd.items() if k not in frozen}
            path = self.ckpt_layer_path(save_dir, i)
            (checkpoint_engine.save(sd, path) if checkpoint_engine is not None else torch.save(sd, path))

    def load_state_dir(self, load_dir, checkpoint_engine=None, strict=True):
        for i, f in enumerate(self.forward_funcs):
            if not isinstance(f, nn.Module) or not list(f.state_dict().keys()):
                continue
            path = self.ckpt_layer_path(load_dir, i)
            sd = torch.load(path, map_location="cpu", weights_only=True)
            f.load_state_dict(sd, strict=strict)
        self._synchronize_tied_weights()


__all__ = ["LayerSpec", "TiedLayerSpec", "PipelineModule", "ProcessTopology", "partition_uniform",
           "partition_balanced"]
