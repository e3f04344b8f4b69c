"""ZeRO stage 3: parameters, gradients and optimizer state partitioned over the data-parallel group.

Parity: reference runtime/zero/stage3.py:128 ``DeepSpeedZeroOptimizer_Stage3`` (reduce-scatter of IPG
grads :1305-1478, step :2112-2174), runtime/zero/partitioned_param_coordinator.py:63 (trace-based
prefetch :285-421, release :425) and runtime/zero/parameter_offload.py:89 (module hooks :244-491).

MI355X-first design (not a port of the per-parameter coordinator):
* The fetch granule is a *module unit* -- e.g. one transformer block -- stored as ONE flat bit16
  buffer (``flat.FlatUnit``). A fetch is ONE ``all_gather_into_tensor`` of ~0.4 GB for a Llama-3-8B
  block (vs. hundreds of per-parameter gathers), and the backward reduction is ONE
  ``reduce_scatter_tensor``. Message sizes this large run RCCL at full xGMI bandwidth.
* Three HIP streams: compute, all-gather (prefetch ``prefetch_depth`` units ahead in the recorded
  forward order, reversed in backward) and reduce-scatter, so parameter traffic, gradient traffic
  and GEMMs overlap. Freed parameter memory goes back to PyTorch's caching allocator through
  ``storage.resize_(0)`` with ``record_stream`` fencing (no host sync).
* Units smaller than ``param_persistence_threshold`` (norm weights, biases) stay gathered; with a
  single rank every unit is persistent, so ZeRO-3 on one GPU has zero gather/release overhead.
* Optional Shuffle-exchange slices (the fork's feature extended to stage 3): partitioning inside
  a slice, bit16 chunk averaging across slices after each step.
* ZeRO++ (reference partition_parameters.py:824-863, coalesced_collectives.py:31-155,
  groups.py:692-749): qwZ all-gathers int8 shards + per-group scales (quantized once per step,
  dequantized by a HIP kernel into the unit buffer); qgZ replaces the reduce-scatter by an int8/int4
  all-to-all whose receive side dequantizes and reduces the W chunks in one kernel; hpZ keeps a
  secondary shard per intra-node group (captured from the forward gather) so backward re-gathers
  only inside that group.
"""
import torch
import torch.nn as nn

from ... import comm as dist
from ...accelerator import get_accelerator
from ...utils.logging import log_dist
from .base import ZeroOptimizerBase
from .flat import FlatUnit
from .partition_parameters import release_construction_partition
from .shuffle_exchange import ShuffleExchange, SliceTopology
from ..torch_autocast import unit_comm_dtype

RELEASED, INFLIGHT, AVAILABLE = 0, 1, 2


def discover_units(module, unit_classes=None):
    """Module units: elements of ModuleLists (or modules whose class name is in `unit_classes`),
    plus every other child that owns parameters; the root keeps any params owned directly."""
    units = []
    covered = set()

    def has_list(m):
        return any(isinstance(c, nn.ModuleList) for c in m.modules())

    def has_params(m):
        return any(True for _ in m.parameters())

    def add(name, m, own_only=False):
        ps = list(m.parameters(recurse=not own_only))
        ps = [p for p in ps if id(p) not in covered]
        if ps:
            units.append((name + ("#own" if own_only else ""), m))
            covered.update(id(p) for p in ps)

    def visit(m, prefix):
        for name, child in m.named_children():
            full = f"{prefix}.{name}" if prefix else name
            if unit_classes:
                if type(child).__name__ in unit_classes:
                    add(full, child)
                else:
                    visit(child, full)
                    add(full, child, own_only=True)
            elif isinstance(child, nn.ModuleList):
                for i, el in enumerate(child):
                    if has_params(el):
                        add(f"{full}.{i}", el)
            elif has_list(child):
                visit(child, full)
                add(full, child, own_only=True)
            elif has_params(child):
                add(full, child)

    visit(module, "")
    root_own = [p for p in module.parameters(recurse=False) if id(p) not in covered]
    if root_own:
        units.append(("#root", module))
    return units


class _BwdHook(torch.autograd.Function):
    """Identity in forward; in backward, gathers the unit before its backward kernels run."""

    @staticmethod
    def forward(ctx, mgr, fg, *args):
        ctx.mgr, ctx.fg = mgr, fg
        return tuple(a.view_as(a) for a in args)

    @staticmethod
    def backward(ctx, *grads):
        ctx.mgr._pre_backward(ctx.fg)
        return (None, None) + grads


class _FetchGroup:
    def __init__(self, idx, name, module, own_only):
        self.idx, self.name, self.module, self.own_only = idx, name, module, own_only
        self.units = []


class ZeroStage3Optimizer(ZeroOptimizerBase):
    def __init__(self, module, init_optimizer, *, loss_scaler, clip_grad=0.0, dp_ranks=None, dp_group=None,
                 prefetch_depth=2, param_persistence_threshold=100_000, communication_data_type=None,
                 unit_classes=None, shuffle_exchange_cfg=None, mp_group=None, timers=None, mics_shard_size=-1,
                 average_master=False, host_step=None, offload_param=False, quantized_weights=False,
                 quantized_gradients=False, hpz_partition_size=1, quant_group_size=128, grad_quant_bits=8,
                 max_reuse_distance=1_000_000_000, max_live_parameters=1_000_000_000, defer_reduce=False,
                 retain_params=False, loco_param=None, prefetch_bucket_size=None,
                 model_persistence_threshold=2**63 - 1, param_swap=None, quantized_nontrainable=False):
        acc = get_accelerator()
        device = torch.device(acc.current_device_name())
        self.module = module
        dp_ranks = list(dp_ranks) if dp_ranks is not None else list(range(dist.get_world_size()))
        se = shuffle_exchange_cfg
        S = len(dp_ranks)
        if se is not None and se.enabled:
            S = se.slice_count
        elif mics_shard_size and mics_shard_size > 0:
            S = mics_shard_size  # MiCS: shard inside groups of mics_shard_size, replicate across
        self.topo = SliceTopology(dp_ranks, S)
        self.mics = bool((mics_shard_size or -1) > 0 and not (se is not None and se.enabled) and self.topo.num_slices > 1)
        self.se = None
        if se is not None and se.enabled and self.topo.num_slices > 1:
            self.se = ShuffleExchange(self.topo, method=se.method, rings=se.rings, shuffle_step=se.shuffle_step,
                                      seed=se.seed, gossip_p=se.gossip_p, average_master=average_master)
        if self.mics:
            self._mics_replica = self.topo.offset_groups(range(self.topo.num_slices))[0]
        part_group = self.topo.slice_group if self.topo.S > 1 else None
        super().__init__(init_optimizer, loss_scaler, clip_grad, part_group,
                         overflow_group=dp_group if self.se is not None else None, mp_group=mp_group,
                         device=device)
        self.host_step = host_step
        # ZeRO-Infinity parameter offload: partitioned bit16 shards live in pinned host memory and
        # are DMA'd in on the all-gather stream at fetch time
        self.offload_param = bool(offload_param)
        if self.se is not None:  # host-resident (offload_param) shards are averaged through device buffers
            self.se.comm_device = device
        # offload_param.device = nvme: non-persistent shards live in a swap file (ZeRO-Infinity),
        # cached in a few pinned buffers (runtime/swap_tensor/partitioned_param_swapper.py)
        self.pswap = None
        if param_swap is not None:
            if host_step is None:
                raise ValueError("offload_param.device=nvme needs offload_optimizer (cpu or nvme): the "
                                 "optimizer step writes the updated shards on the host")
            if quantized_weights:
                raise ValueError("offload_param.device=nvme does not combine with zero_quantized_weights")
            from ..swap_tensor.partitioned_param_swapper import AsyncPartitionedParameterSwapper
            self.pswap = AsyncPartitionedParameterSwapper(**param_swap)
            self.offload_param = True
        self.S = self.topo.S
        # ZeRO++ knobs
        self.qwz = bool(quantized_weights) and self.S > 1
        self.qgz = bool(quantized_gradients) and self.S > 1
        self.loco = dict(loco_param) if (loco_param and self.qgz) else None  # zeropp_loco_param
        self._loco_idx = 0
        self.qgroup = int(quant_group_size)
        self.gbits = int(grad_quant_bits)
        # zero_quantized_nontrainable_weights: frozen shards stored int8 + group scales (quant.hip),
        # dequantized by the gather (reference stage3.py:1558, partition_parameters.py:1685,1769)
        self.quant_frozen = bool(quantized_nontrainable)
        self.hpz = int(hpz_partition_size or 1)
        self.hpz_group = None
        if self.hpz > 1 and self.S > self.hpz:
            assert self.S % self.hpz == 0, "zero_hpz_partition_size must divide the partition size"
            ranks = self.topo.dp_ranks  # every rank creates every block's group (collective)
            me = dist.get_rank()
            for i in range(0, len(ranks), self.hpz):
                blk = ranks[i:i + self.hpz]
                g = dist.new_group(blk)
                if me in blk:
                    self.hpz_group, self.hpz_rank = g, blk.index(me)
        else:
            self.hpz = 1
        self.prefetch_depth = max(0, int(prefetch_depth))
        # stage3_prefetch_bucket_size (when given instead of prefetch_depth): prefetch the next
        # fetch groups until this many elements are in flight (at least one group)
        self.prefetch_numel = int(prefetch_bucket_size) if prefetch_bucket_size else None
        self.persist_thr = int(param_persistence_threshold)
        self.tracer = None          # compile/profiler.ScheduleTracer while the schedule compiler traces
        self.prefetch_plan = None   # compiled prefetch trigger table (apply_compile_plan)
        self.compile_plan = None
        # stage3_model_persistence_threshold: cap on the total elements kept persistent
        self.model_persist_thr = int(model_persistence_threshold)
        self._persist_total = 0
        self.max_reuse_distance = int(max_reuse_distance)
        self.max_live_parameters = int(max_live_parameters)
        self._kept_numel = 0
        self.comm_dtype = communication_data_type
        self.timers = timers
        # side streams only where they carry work: with one rank and resident parameters there are
        # no gathers or reduce-scatters, and every extra stream competes for the few HW queues
        # (GPU_MAX_HW_QUEUES) -- a stream sharing the compute stream's queue serialises with it
        comm = self.S > 1 or self.offload_param or self.pswap is not None
        self.ag_stream = acc.named_stream("zero3_allgather") if acc.gpu and comm else None
        self.rs_stream = acc.named_stream("zero3_reduce") if acc.gpu and comm else None
        # gradient reduce-scatters (and the qgZ all-to-alls) get their own communicator over the
        # slice ranks: on the all-gathers' communicator RCCL would queue them behind the backward
        # prefetch gathers (one internal stream per communicator), whatever HIP stream issues them
        self.reduce_group = self.topo.make_reduce_groups() if self.S > 1 else None
        self._in_bwd = False
        self._hooks = []
        self.fgroups = []
        self.param_unit = {}
        # frozen (requires_grad=False) parameters: gather-only units -- partitioned bit16 (or int8)
        # shard, fetched and released with their module, no gradient / master / optimizer state
        self.frozen_unit = {}
        self.frozen_units = []
        self._bwd_frozen = []
        self._build(unit_classes)
        self._init_master()
        self._register()
        for units in self.units:  # accumulators start zeroed: every slot counts as written
            for u in units:
                u.acc_valid = [True] * len(u.params)
                u.rs_valid = True
        # deferred reduce-scatter (zero_optimization.stage3_defer_reduce): units keep an fp32
        # gradient sum across micro-steps (4 B/param of HBM) and reduce-scatter at the boundary
        self.defer_reduce = bool(defer_reduce) and self.S > 1 and not self.qgz
        # retain gathered units across the micro-steps of one optimizer step (weights cannot change
        # before the step): one all-gather per unit per step instead of one or two per micro-step
        self.retain_params = bool(retain_params) and self.S > 1
        self._boundary = True
        if self.defer_reduce:
            for units in self.units:
                for u in units:
                    u.staging_dtype = torch.float32
        self.trace = [fg.idx for fg in self.fgroups]
        self._observed = []
        n_units = sum(len(u) for u in self.units)
        n_persist = sum(1 for units in self.units for u in units if u.persistent)
        log_dist(f"ZeRO-3: {len(self.fgroups)} fetch groups / {n_units} units ({n_persist} persistent), "
                 f"partition={self.S}, slices={self.topo.num_slices}, prefetch_depth={self.prefetch_depth}, "
                 f"mics={self.mics}, shuffle_exchange={se.method if self.se is not None else 'off'}, "
                 f"defer_reduce={self.defer_reduce}, retain_params={self.retain_params}", ranks=[0])

    # ------------------------------------------------------------------------------------- layout
    def _build(self, unit_classes):
        group_of = {}
        for g, pg in enumerate(self.optimizer.param_groups):
            for p in pg["params"]:
                group_of[id(p)] = g
        self.units = [[] for _ in self.optimizer.param_groups]
        for fi, (name, mod) in enumerate(discover_units(self.module, unit_classes)):
            own_only = name.endswith("#own") or name == "#root"
            allp = list(mod.parameters(recurse=not own_only))
            params = [p for p in allp if p.requires_grad and id(p) in group_of and p not in self.param_unit]
            # frozen weights (a LoRA base model, frozen embeddings) are owned by ZeRO-3 too: without
            # this a zero.Init-partitioned frozen parameter has no data at all, and one built whole
            # would stay whole on every rank (reference partitioned_param_coordinator.py:300,437,544
            # fetches every parameter of a submodule, trainable or not)
            frozen = [p for p in allp if not p.requires_grad and p not in self.frozen_unit
                      and getattr(p, "allreduce", True) is not False]
            if not params and not frozen:
                continue
            fg = _FetchGroup(len(self.fgroups), name, mod, own_only)
            by_group = {}
            for p in params:
                by_group.setdefault(group_of[id(p)], []).append(p)
            for g, plist in sorted(by_group.items()):
                u = self._make_unit(plist, f"{name}/g{g}", fg)
                self.units[g].append(u)
                fg.units.append(u)
                for p in plist:
                    self.param_unit[p] = u
            by_dt = {}
            for p in frozen:  # one flat buffer per dtype (e.g. an fp8-coded LoRA base next to a bf16 bias)
                by_dt.setdefault(p.dtype, []).append(p)
            for dt, plist in by_dt.items():
                u = self._make_unit(plist, f"{name}/frozen" + ("" if len(by_dt) == 1 else f"/{dt}"), fg, frozen=True)
                fg.units.append(u)
                self.frozen_units.append(u)
                for p in plist:
                    self.frozen_unit[p] = u
            self.fgroups.append(fg)
        # external parameters: a module that uses a parameter owned by another unit (tied
        # embeddings / LM head, or register_external_parameter) fetches that unit too (reference
        # partition_parameters.py register_external_parameter, parameter_offload.py external params)
        fg_of = {id(fg.module): fg for fg in self.fgroups}
        owner = dict(self.frozen_unit)
        owner.update(self.param_unit)

        def scan(mod, name, cover):
            fg = fg_of.get(id(mod))
            here = fg if fg is not None else cover  # the fetch group whose hook runs around mod
            ext = list(getattr(mod, "_sxe_external_params", []))
            ext += [p for p in mod.parameters(recurse=False)
                    if p in owner and owner[p].fg is not here]
            ext_units = []
            for p in ext:
                u = owner.get(p)
                if u is not None and u not in ext_units and (here is None or u not in here.units):
                    ext_units.append(u)
            if ext_units:
                if fg is None:
                    fg = _FetchGroup(len(self.fgroups), (name or "#root") + "#external", mod, True)
                    self.fgroups.append(fg)
                    fg_of[id(mod)] = fg
                fg.units.extend(ext_units)
            nxt = cover if (fg is not None and fg.own_only) else (fg if fg is not None else cover)
            for cname, child in mod.named_children():
                scan(child, f"{name}.{cname}" if name else cname, nxt)
        scan(self.module, "", None)
        # any trainable param not under a discovered module (should not happen) -> root unit
        rest = [p for pg in self.optimizer.param_groups for p in pg["params"] if p.requires_grad and p not in self.param_unit]
        if rest:
            fg = _FetchGroup(len(self.fgroups), "#rest", self.module, True)
            for p in rest:
                u = self._make_unit([p], "#rest", fg)
                u.persistent = True
                self.units[group_of[id(p)]].append(u)
                fg.units.append(u)
                self.param_unit[p] = u
            self.fgroups.append(fg)

    def _make_unit(self, params, name, fg, frozen=False):
        dtype = params[0].dtype
        u = FlatUnit(params, self.S, self.topo.offset, dtype, self.device, name=name, materialize_full=False)
        u.comm_dtype = unit_comm_dtype(params)  # torch_autocast: bf16 reduce-scatter when every param is marked
        u.fg = fg
        u.owner = self
        u.frozen = frozen
        u.frozen_q = False
        u.persistent = (self.S == 1 and not self.offload_param) or (
            u.numel < self.persist_thr and self._persist_total + u.numel <= self.model_persist_thr)
        if u.persistent:
            self._persist_total += u.numel
        flat = torch.zeros(u.padded, dtype=dtype, device=self.device)
        with torch.no_grad():
            for p, o, n in zip(u.params, u.offsets, u.numels):
                if hasattr(p, "ds_tensor_full"):
                    # zero.Init construction partition: gather this one parameter, then drop the
                    # per-parameter chunk (the unit shard below replaces it)
                    flat[o:o + n].copy_(p.ds_tensor_full().reshape(-1))
                    release_construction_partition(p)
                else:
                    flat[o:o + n].copy_(p.data.reshape(-1))
        u.flat = flat
        u.link_params()
        if u.persistent:
            u.shard = flat[u.lo:u.hi]
            u.state = AVAILABLE
        else:
            if self.pswap is not None and not frozen:
                self.pswap.register(u, flat[u.lo:u.hi].cpu())
                u.shard = None
                u.swap = self.pswap
            elif self.offload_param:
                if flat.is_cuda:
                    from .offload import pinned_empty  # exact-size pinned (no power-of-2 rounding)
                    u.shard = pinned_empty(u.chunk, dtype)
                else:
                    u.shard = torch.empty(u.chunk, dtype=dtype)
                u.shard.copy_(flat[u.lo:u.hi])
            else:
                u.shard = flat[u.lo:u.hi].clone()
            u.flat.untyped_storage().resize_(0)
            u.unlink_params()
            u.state = RELEASED
        u.event = None
        u.keep = False
        u.qshard = None
        u.sec_shard, u.sec_valid = None, False
        for p in params:
            p.ds_unit = u
        if frozen and self.quant_frozen:
            self._quantize_frozen(u)
        return u

    def _quantize_frozen(self, u):
        """Store a frozen unit's shard as int8 + fp32 group scales (half the bytes of bf16); the
        gather all-gathers the int8 shards and dequantizes into the unit buffer. Resident units
        (one rank, small units, host-resident shards) keep bit16."""
        if (u.persistent or u.frozen_q or self.S == 1 or u.swap is not None or u.shard.device != self.device
                or u.dtype not in (torch.bfloat16, torch.float16, torch.float32)):
            return False
        self._quantize_shard(u)
        u.shard = None
        u.frozen_q = True
        return True

    def quantize_nontrainable_params(self):
        """Quantize every frozen unit that is still stored in bit16 (reference stage3.py:1558: after
        ``zero_quantized_nontrainable_weights`` was switched on, or frozen units were added).
        Returns the number of units quantized."""
        if not self.quant_frozen:
            log_dist("quantize_nontrainable_params(): zero_quantized_nontrainable_weights is off, nothing to do",
                     ranks=[0])
            return 0
        self.wait_params()
        return sum(1 for u in self.frozen_units if self._quantize_frozen(u))

    def frozen_state_dict(self, keep=True):
        """{param: full host tensor} of every frozen parameter (a collective: gathers each frozen
        unit in turn, then releases it). Ranks with ``keep=False`` take part without a copy."""
        out = {}
        self.wait_params()
        for u in self.frozen_units:
            was = u.state
            if not u.persistent:
                self._fetch_unit(u)
            if keep:
                for p in u.params:
                    out[p] = p.detach().cpu().clone()
            if not u.persistent and was == RELEASED:
                self._release_unit(u)
        return out

    # -------------------------------------------------------------------------------------- hooks
    def _register(self):
        self._module_hooks = []
        for fg in self.fgroups:
            if fg.name == "#rest":
                continue
            self._module_hooks.append(fg.module.register_forward_pre_hook(self._make_pre(fg)))
            self._module_hooks.append(fg.module.register_forward_hook(self._make_post(fg)))
        self._hooks.extend(self._module_hooks)
        for p, u in self.param_unit.items():
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_grad_hook(u)))
            # fused weight-grad GEMMs (ops/linear.py) write straight into the unit's buffers
            p._sxe_grad_target = self._grad_target
            p._sxe_grad_done = self._grad_done
            p._sxe_grad_defer = self._grad_defer

    def _grad_defer(self, p):
        """May a weight-gradient producer hold this micro-step's contribution and write it with a
        later one (ops/mlp.py weight_grad_tn)? Before the accumulation boundary, for a persistent
        single-rank unit: its fp32 accumulator is read by nothing until the optimizer step."""
        u = self.param_unit.get(p)
        return not self._boundary and u is not None and u.persistent and self.S == 1

    # ---------------------------------------------------------------------- FX graph mode
    def enter_graph_mode(self):
        """Hand fetch / release to a compiled graph (compile/fx_zero3.py): the module hooks go, and
        a released unit keeps its parameters linked as full-shape views of its flat buffer whose
        STORAGE is freed (``resize_(0)``) -- the traced graph sees fixed parameter shapes, and a
        gather re-allocates the same storage in place, so the views (and any tensors autograd saved
        from them) become valid again."""
        self.graph_mode = True
        for h in getattr(self, "_module_hooks", []):
            h.remove()
        self._module_hooks = []
        for units in self.units:
            for u in units:
                if u.state == RELEASED:  # relink as views (storage stays freed)
                    u.flat.untyped_storage().resize_(u.padded * u.flat.element_size())
                    u.link_params()
                    u.flat.untyped_storage().resize_(0)
        self.trace = []

    def graph_relink(self):
        """Before a compiled forward: released units show their parameters as full-shape views of the
        freed flat storage again (the shapes the traced graphs were specialised on)."""
        self._in_graph_step = True
        for units in self.units:
            for u in units:
                if getattr(u, "graph_unlinked", False):
                    if u.state == RELEASED:
                        st = u.flat.untyped_storage()
                        st.resize_(u.padded * u.flat.element_size())  # views need in-bounds storage
                        u.link_params()
                        st.resize_(0)
                    u.graph_unlinked = False

    def graph_unlink(self):
        """After a compiled step (backward done, or a no-grad forward): released parameters read as
        empty tensors (numel 0) -- as in eager ZeRO-3 -- instead of full-shape views over freed
        storage that a read outside GatheredParameters would dereference."""
        self._in_graph_step = False
        for units in self.units:
            for u in units:
                if u.state == RELEASED and not u.persistent and not getattr(u, "graph_unlinked", False):
                    u.unlink_params()
                    u.graph_unlinked = True

    def gather_all_for_trace(self):
        """Materialise every unit (Dynamo fake-ifies the parameters when it traces)."""
        for fg in self.fgroups:
            self._fetch(fg, wait=True)

    def grad_ready(self, p):
        """A gradient delivered by a compiled graph's reduce node: run the per-parameter hook."""
        u = self.param_unit.get(p)
        if u is not None:
            self._make_grad_hook(u)(p)

    def _grad_target(self, p):
        u = self.param_unit[p]
        i = u.param_index[id(p)]
        o, n = u.offsets[i], u.numels[i]
        if u.persistent and self.S == 1:
            return u.grad[o:o + n].view(p.ds_shape), u.acc_valid[i]
        if u.staging is None:
            u.staging = torch.empty(u.padded, dtype=u.staging_dtype or u.dtype, device=u.device)
            if u.padded > u.numel:
                u.staging[u.numel:].zero_()
        return u.staging[o:o + n].view(p.ds_shape), u.filled[i] or u.carry

    def _grad_done(self, p):
        u = self.param_unit[p]
        i = u.param_index[id(p)]
        if u.persistent and self.S == 1:
            u.filled[i] = True
            u.acc_valid[i] = True
            return
        if not u.filled[i]:
            u.filled[i] = True
            u.pending -= 1
        if u.pending == 0:
            self._reduce_unit(u)
            if not u.persistent and self._in_bwd:
                self._release_unit(u)

    def _make_pre(self, fg):
        def pre(mod, args):
            if not self._in_bwd:
                self._observed.append(fg.idx)
            if self.host_step is not None:
                self.host_step.wait_units(fg.units)  # asynchronous host update (zero/offload.py)
            for u in fg.units:
                self.wait_step_unit(u)  # overlapped device update (zero/base.py)
            self._fetch(fg, wait=True)
            self._prefetch_after(fg, backward=self._in_bwd)
            if self.tracer is not None and not self._in_bwd:
                self.tracer.on_fwd_begin(fg)
        return pre

    def _make_post(self, fg):
        def post(mod, args, out):
            if self.tracer is not None and not self._in_bwd:
                self.tracer.on_fwd_end(fg)
            if torch.is_grad_enabled():  # frozen-only groups too: their backward reads the weights
                out = self._wrap_outputs(fg, out)
            if not self._in_bwd and not (torch.is_grad_enabled() and self._keep_for_backward(fg)):
                self._release(fg)
            return out
        return post

    def _wrap_outputs(self, fg, out):
        if isinstance(out, torch.Tensor):
            if out.requires_grad:
                return _BwdHook.apply(self, fg, out)[0]
            return out
        if isinstance(out, (tuple, list)):
            idx = [i for i, t in enumerate(out) if isinstance(t, torch.Tensor) and t.requires_grad]
            if not idx:
                return out
            wrapped = _BwdHook.apply(self, fg, *[out[i] for i in idx])
            lst = list(out)
            for i, w in zip(idx, wrapped):
                lst[i] = w
            return type(out)(lst) if isinstance(out, tuple) else lst
        if isinstance(out, dict):
            keys = [k for k, t in out.items() if isinstance(t, torch.Tensor) and t.requires_grad]
            if not keys:
                return out
            wrapped = _BwdHook.apply(self, fg, *[out[k] for k in keys])
            new = type(out)(out)
            for k, w in zip(keys, wrapped):
                new[k] = w
            return new
        return out

    def _is_last_forward(self, fg):
        return bool(self.trace) and self.trace[-1] == fg.idx

    def _reuse_distances(self):
        """Per fetch group: gathered numel traversed between its forward use and its backward
        re-use (the later forward groups, then the same groups again in reverse), i.e. the
        reference's reuse distance (partitioned_param_coordinator.py:529-559) on our unit trace."""
        key = tuple(self.trace)
        if getattr(self, "_reuse_key", None) != key:
            size = {fg.idx: sum(u.padded for u in fg.units if not u.persistent) for fg in self.fgroups}
            dist_, acc = {}, 0
            for i in reversed(self.trace):
                dist_[i] = 2 * acc
                acc += size.get(i, 0)
            self._reuse, self._reuse_key, self._fg_numel = dist_, key, size
        return self._reuse

    def _keep_for_backward(self, fg):
        """Keep a forward-gathered group resident for its backward re-use when its reuse distance is
        below ``max_reuse_distance`` and the resident budget ``max_live_parameters`` allows it. With
        288 GB of HBM per GPU a whole 8B model fits (16 GB bf16), which removes the backward
        all-gather (one third of ZeRO-3's per-micro-step traffic)."""
        if self._is_last_forward(fg):
            return True
        if self.max_reuse_distance <= 0 or self.S == 1:
            return False
        d = self._reuse_distances().get(fg.idx)
        n = self._fg_numel.get(fg.idx, 0)
        if d is None or d >= self.max_reuse_distance or self._kept_numel + n > self.max_live_parameters:
            return False
        self._kept_numel += n
        return True

    def _make_grad_hook(self, unit):
        def hook(p):
            if p.grad is None or getattr(p, "_sxe_grad_partial", False):
                return  # partial tile gradient: keep summing in .grad until the last tile
            if unit.persistent and self.S == 1:
                i = unit.param_index[id(p)]
                o, n = unit.offsets[i], unit.numels[i]
                if unit.acc_valid[i]:
                    unit.grad[o:o + n].add_(p.grad.reshape(-1))
                else:
                    unit.grad[o:o + n].copy_(p.grad.reshape(-1))
                    unit.acc_valid[i] = True
                if not unit.filled[i]:
                    unit.filled[i] = True
                    unit.pending -= 1
                p.grad = None
                return
            done = unit.stage_grad(p, p.grad)
            p.grad = None
            if done:
                self._reduce_unit(unit)
                if not unit.persistent and self._in_bwd and not getattr(self, "graph_mode", False):
                    self._release_unit(unit)
        return hook

    # ------------------------------------------------------------------------------ fetch/release
    def _launch_gather(self, u):
        if self.host_step is not None:
            self.host_step.wait_unit(u)  # the shard is final once the host update reached it
        cur = torch.cuda.current_stream() if u.flat.is_cuda else None  # shard may be host-resident (offload_param)
        st = self.ag_stream
        if st is not None:
            self.wait_step_unit(u, st)
            st.wait_stream(cur)
        elif cur is not None:
            self.wait_step_unit(u)
        with get_accelerator().stream(st):
            u.flat.untyped_storage().resize_(u.padded * u.flat.element_size())
            if not getattr(self, "graph_mode", False) or getattr(u, "graph_unlinked", False):
                u.link_params()
                u.graph_unlinked = False
            swapped = u.swap is not None
            src = u.swap.acquire(u) if swapped else u.shard
            if src is None:  # int8 frozen shard: the quantized gather below reads u.qshard
                src = u.flat
            elif src.device != u.flat.device:
                src = src.to(u.flat.device, non_blocking=True)
                if st is not None:
                    src.record_stream(st)
            if swapped:  # the pinned swap buffer may be reused once this H2D copy has run
                ev = None
                if u.flat.is_cuda:
                    ev = torch.cuda.Event()
                    ev.record(st if st is not None else cur)
                u.swap.release(u, ev)
            t0 = self.tracer.gather_begin(u, st) if self.tracer is not None else None
            if self.S == 1:
                u.flat.copy_(src)
            elif self.hpz > 1 and self._in_bwd and u.sec_valid:
                # hpZ: backward re-gather inside the intra-node group from the secondary shards
                dist.all_gather_into_tensor(u.flat, u.sec_shard, group=self.hpz_group)
            elif self.qwz or u.frozen_q:
                self._quantized_gather(u, st)
            else:
                dist.all_gather_into_tensor(u.flat, src, group=self.topo.slice_group)
            if t0 is not None:
                self.tracer.gather_end(u, st, t0)
            if st is not None:
                u.event = torch.cuda.Event()
                u.event.record(st)
        u.state = INFLIGHT

    def _qgroup(self, u):
        return self.qgroup if u.chunk % self.qgroup == 0 else 64

    def _quantize_shard(self, u):
        from ...ops.quantizer import quantize
        q, sc = quantize(u.shard, self._qgroup(u), 8)
        u.qshard = (q, sc)

    def _quantized_gather(self, u, st):
        """qwZ: all-gather int8 shards + fp32 group scales, dequantize into the unit buffer."""
        from ...ops.quantizer import dequantize
        if u.qshard is None:
            self._quantize_shard(u)
        q, sc = u.qshard
        qa = torch.empty(q.numel() * self.S, dtype=q.dtype, device=q.device)
        sa = torch.empty(sc.numel() * self.S, dtype=sc.dtype, device=sc.device)
        dist.all_gather_into_tensor(qa, q, group=self.topo.slice_group)
        dist.all_gather_into_tensor(sa, sc, group=self.topo.slice_group)
        dequantize(qa, sa, self._qgroup(u), 8, out=u.flat)
        if st is not None:
            qa.record_stream(st)
            sa.record_stream(st)

    def _fetch_unit(self, u):
        if u.state == RELEASED:
            self._launch_gather(u)
        if u.state == INFLIGHT:
            if u.event is not None:
                cur = torch.cuda.current_stream()
                cur.wait_event(u.event)
                u.flat.record_stream(cur)
            u.state = AVAILABLE

    def _fetch(self, fg, wait=True):
        for u in fg.units:
            if u.persistent:
                continue
            if u.state == RELEASED:
                self._launch_gather(u)
            if wait and u.state == INFLIGHT:
                if u.event is not None:
                    cur = torch.cuda.current_stream()
                    cur.wait_event(u.event)
                    u.flat.record_stream(cur)
                u.state = AVAILABLE

    def _release_unit(self, u):
        if u.persistent or u.keep or u.state == RELEASED or getattr(self, "_hold", False):
            return
        if getattr(self, "retain_params", False) and (not self._in_bwd or not self._boundary):
            return  # still valid until the optimizer step: only the boundary backward releases
        if u.state == INFLIGHT and u.event is not None:
            torch.cuda.current_stream().wait_event(u.event)
        if self.hpz > 1 and not self._in_bwd and not u.sec_valid:
            n = u.padded // self.hpz
            if u.sec_shard is None:
                u.sec_shard = torch.empty(n, dtype=u.flat.dtype, device=u.flat.device)
            u.sec_shard.copy_(u.flat[self.hpz_rank * n:(self.hpz_rank + 1) * n])
            u.sec_valid = True
        u.flat.untyped_storage().resize_(0)
        if not getattr(self, "graph_mode", False):
            u.unlink_params()
        elif not getattr(self, "_in_graph_step", False):  # a gather outside a compiled step
            u.unlink_params()
            u.graph_unlinked = True
        u.state = RELEASED

    def _release(self, fg):
        for u in fg.units:
            self._release_unit(u)

    def _prefetch_after(self, fg, backward):
        if self.prefetch_depth == 0 or (self.S == 1 and not self.offload_param):
            return
        if self.prefetch_plan is not None:  # compiled schedule (compile/passes.py prefetch)
            for j in self.prefetch_plan["bwd" if backward else "fwd"].get(fg.idx, ()):
                self._fetch(self.fgroups[j], wait=False)
            return
        order = list(reversed(self.trace)) if backward else self.trace
        if fg.idx not in order:
            return
        i = order.index(fg.idx)
        if self.prefetch_numel is not None:
            acc = 0
            for j in order[i + 1:]:
                if acc >= self.prefetch_numel:
                    break
                nxt = self.fgroups[j]
                self._fetch(nxt, wait=False)
                acc += sum(u.padded for u in nxt.units if not u.persistent)
            return
        for j in order[i + 1:i + 1 + self.prefetch_depth]:
            self._fetch(self.fgroups[j], wait=False)
        if self.pswap is not None:
            # NVMe read-ahead beyond the gather window, into whatever swap buffers are free now
            for j in order[i + 1 + self.prefetch_depth:i + 1 + 2 * self.prefetch_depth + 2]:
                for u in self.fgroups[j].units:
                    if u.swap is not None and u.state == RELEASED:
                        self.pswap.prefetch(u)

    def _pre_backward(self, fg):
        self._in_bwd = True
        if self._bwd_frozen:
            # frozen units get no gradient hook to release them: the previous group's backward has
            # run once the next group's output gradient exists
            keep = [u for u in self._bwd_frozen if u in fg.units]
            for u in self._bwd_frozen:
                if u not in keep:
                    self._release_unit(u)
            self._bwd_frozen = keep
        self._fetch(fg, wait=True)
        self._bwd_frozen.extend(u for u in fg.units if u.frozen and not u.persistent and u not in self._bwd_frozen)
        self._prefetch_after(fg, backward=True)
        if self.tracer is not None:
            self.tracer.on_bwd_begin(fg)

    # ------------------------------------------------------------------------------ grad reduction
    def _reduce_unit(self, u):
        if self.defer_reduce and not self._boundary:
            # 288 GB HBM: keep the unit's fp32 gradient sum local across the micro-steps of one
            # optimizer step and reduce-scatter it once, at the accumulation boundary (1/GAS of
            # the per-micro-step reduce-scatter traffic over xGMI)
            u.carry = True
            return
        u.carry = False
        st = u.staging
        u.staging = None
        cur = torch.cuda.current_stream() if st.is_cuda else None
        rs = self.rs_stream
        if rs is not None:
            rs.wait_stream(cur)
        with get_accelerator().stream(rs):
            want = (u.comm_dtype if self.S > 1 else None) or self.comm_dtype or (u.dtype if self.defer_reduce else None)
            send = st if (want is None or st.dtype == want) else st.to(want)
            if self.S == 1:
                self._accumulate(u, send, 1.0)
            elif self.qgz and not self.mics:
                self._quantized_reduce_scatter(u, st)
            else:
                out = torch.empty(u.chunk, dtype=send.dtype, device=send.device)
                dist.reduce_scatter_tensor(out, send, group=self.reduce_group)
                if self.mics:
                    dist.all_reduce(out, group=self._mics_replica)
                    self._accumulate(u, out, self.sp_scale / (self.S * self.topo.num_slices))
                else:
                    self._accumulate(u, out, self.sp_scale / self.S)
                if rs is not None:
                    out.record_stream(rs)
            if rs is not None:
                st.record_stream(rs)
                send.record_stream(rs)

    def _accumulate(self, u, x, alpha):
        """u.grad += alpha * x, or = alpha * x for the first reduction of the step (no memset of
        the fp32 accumulators between steps, see zero_grad_buffers)."""
        if u.rs_valid:
            u.grad.add_(x, alpha=alpha)
        else:
            torch.mul(x, alpha, out=u.grad) if x.dtype == u.grad.dtype else u.grad.copy_(x).mul_(alpha)
            u.rs_valid = True

    def zero_grad_buffers(self):
        """Mark the fp32 gradient accumulators stale instead of zeroing them (a 32 GB memset per
        step on an 8B model at dp=1): each slot's first write of the next step overwrites (GEMMs
        with beta = 0, copy_ in the hooks, assignment after the reduce-scatter) and slots no
        gradient reached are zeroed right before the step (_zero_stale)."""
        for units in self.units:
            for u in units:
                u.acc_valid = [False] * len(u.params)
                u.rs_valid = False
                for p in u.params:
                    p.__dict__.pop("_sxe_bstash", None)  # a partial accumulation goes with the rest

    def _zero_stale(self):
        if self.host_step is not None:
            self.host_step.wait_grad_mirror()  # the async host update's D2H may still read u.grad
        for units in self.units:
            for u in units:
                if u.persistent and self.S == 1:
                    for i, ok in enumerate(u.acc_valid):
                        if not ok:
                            o, n = u.offsets[i], u.numels[i]
                            u.grad[o:o + n].zero_()
                    u.acc_valid = [True] * len(u.params)
                elif not u.rs_valid:
                    u.grad.zero_()
                    u.rs_valid = True

    def _quantized_reduce_scatter(self, u, staging):
        """qgZ: quantize the full gradient unit per destination chunk, all-to-all the packed
        chunks, dequantize + reduce the W received chunks straight into this rank's accumulator."""
        from ...ops.quantizer import dequant_reduce, quantize
        qg = self._qgroup(u)
        if self.loco is not None:
            # LoCo error feedback (reference coalesced_collectives.all_to_all_loco_quant_reduce):
            # quantize grad + err_beta * (previous quantization error) and keep the new error,
            # reset every reset_T reductions; the error buffer is stored in the gradient dtype
            from ...ops.quantizer import loco_quantize
            beta, reset_t = float(self.loco.get("err_beta", 0.8)), int(self.loco.get("reset_T", 1024))
            err = getattr(u, "loco_err", None)
            if self._loco_idx > reset_t:
                err, self._loco_idx = None, 0
            q, sc, new_err = loco_quantize(staging, err, beta, qg, self.gbits)
            u.loco_err = new_err.to(staging.dtype)
            self._loco_idx += 1
        else:
            q, sc = quantize(staging, qg, self.gbits)
        rq, rs = torch.empty_like(q), torch.empty_like(sc)
        dist.all_to_all_single(rq, q, group=self.reduce_group)
        dist.all_to_all_single(rs, sc, group=self.reduce_group)
        dequant_reduce(rq, rs, self.S, qg, self.gbits, u.grad, alpha=self.sp_scale / self.S, accumulate=u.rs_valid)
        u.rs_valid = True
        if self.rs_stream is not None:
            for t in (q, sc, rq, rs):
                t.record_stream(self.rs_stream)

    def forward_prologue(self):
        self._in_bwd = False
        self._observed = []
        self._kept_numel = 0
        if self.tracer is not None:
            self.tracer.on_forward_start()

    def backward_prologue(self):
        self.drain_step()
        if self.host_step is not None:
            self.host_step.before_backward()
        for units in self.units:
            for u in units:
                u.begin_backward()

    def set_gradient_accumulation_boundary(self, flag):
        self._boundary = bool(flag)

    def reduce_gradients(self, pipeline_parallel=False):
        if self._boundary:
            from ...ops.mlp import flush_stashed_wgrad
            for p in self.param_unit:
                if p.__dict__.get("_sxe_bstash") is not None:  # held weight grads the boundary did not consume
                    flush_stashed_wgrad(p)
        for units in self.units:
            for u in units:
                if u.pending > 0:
                    if u.persistent and self.S == 1:
                        continue
                    for i, p in enumerate(u.params):
                        if not u.filled[i] and p.grad is not None:
                            u.stage_grad(p, p.grad)
                            p.grad = None
                    if u.pending > 0:
                        u.fill_missing()
                    self._reduce_unit(u)
                if not u.persistent:
                    self._release_unit(u)
        for u in self.frozen_units:
            if not u.persistent:
                self._release_unit(u)
        self._bwd_frozen = []
        if self._observed and self._observed != self.trace:
            # trace changed (data-dependent control flow): adopt the new order
            seen, order = set(), []
            for i in self._observed:
                if i not in seen:
                    seen.add(i)
                    order.append(i)
            self.trace = order
        self._in_bwd = False
        if self.tracer is not None:
            self.tracer.on_backward_end()

    # ------------------------------------------------------------------------------------------ step
    supports_async_host_step = True
    supports_overlapped_step = True  # zero/base.py _overlapped_update

    def step_unit_order(self):
        return self.host_unit_order()

    def wait_params(self):
        """Nothing in flight across steps on the device (the update runs on the compute stream);
        an asynchronous host-offload update (zero/offload.py) is finished here."""
        self.drain_step()
        if self.host_step is not None:
            self.host_step.wait_all()

    def host_unit_order(self):
        """Units in the order the next forward needs them: the ``#rest`` group (parameters read
        outside any hooked module) first -- after the small resident units the post-step refresh
        all-gathers when the partition has several ranks --, then the recorded forward trace,
        then the rest."""
        seen, out = set(), []
        rest = [fg for fg in self.fgroups if fg.name == "#rest"]
        groups = rest + [self.fgroups[j] for j in self.trace] + list(self.fgroups)
        resident = [u for fg in groups for u in fg.units if (u.persistent or u.keep) and not u.frozen]
        for u in (resident if self.S > 1 else []) + [u for fg in groups for u in fg.units if not u.frozen]:
            if id(u) not in seen:
                seen.add(id(u))
                out.append(u)
        return out

    def step(self, closure=None, lr_kwargs=None):
        self.wait_params()
        if self.rs_stream is not None:
            torch.cuda.current_stream().wait_stream(self.rs_stream)
        if self.se is not None and self.se.method == "Gossip":
            self.se.pre_step([u.shard for units in self.units for u in units])
        self._zero_stale()
        coef, skip = self._grad_norm_and_flags()
        if getattr(self.loss_scaler, "dynamic", False) and self._handle_overflow_host():
            self.zero_grad_buffers()
            return
        self._fused_update(coef, skip)
        self.zero_grad_buffers()
        for fg in self.fgroups:
            if fg.name == "#rest":  # read outside any module hook: final before the next forward
                if self.host_step is not None:
                    self.host_step.wait_units(fg.units)
                for u in fg.units:
                    self.wait_step_unit(u)
        if self.se is not None:
            self.wait_params()
        if self.se is not None:
            self.se.sync([u.shard for units in self.units for u in units], self._device_masters())
        self._refresh_persistent()
        for units in self.units:
            for u in units:
                u.sec_valid = False
                if self.qwz and not u.persistent:
                    self._quantize_shard(u)
        self.global_step += 1
        # start gathering the first units of the next forward now
        for j in self.trace[:self.prefetch_depth]:
            self._fetch(self.fgroups[j], wait=False)

    def _refresh_persistent(self):
        """Rebuild the full copies of the resident units (persistent small parameters, plan-kept
        units) after the step: ONE all-gather of all their shards packed back to back -- a
        Llama-3-8B has ~65 persistent norm-weight units, and as many separate latency-bound
        gathers cost more than the packed message -- then one strided copy per unit from the
        rank-major result into its flat buffer."""
        if self.S == 1:
            return
        units = [u for us in self.units for u in us if u.persistent or (u.keep and u.state == AVAILABLE)]
        if not units:
            return
        # their shards come from the (possibly asynchronous) update: wait for exactly these units,
        # which the update order puts first (host_unit_order), not for the whole update
        if self.host_step is not None:
            self.host_step.wait_units(units)
        for u in units:
            self.wait_step_unit(u)
        if len(units) == 1:
            u = units[0]
            dist.all_gather_into_tensor(u.flat, u.shard, group=self.topo.slice_group)
            return
        total = sum(u.chunk for u in units)
        send = torch.empty(total, dtype=units[0].dtype, device=units[0].flat.device)
        off = 0
        for u in units:
            send[off:off + u.chunk].copy_(u.shard)
            off += u.chunk
        recv = torch.empty(self.S * total, dtype=send.dtype, device=send.device)
        dist.all_gather_into_tensor(recv, send, group=self.topo.slice_group)
        rv = recv.view(self.S, total)
        off = 0
        for u in units:
            u.flat.view(self.S, u.chunk).copy_(rv[:, off:off + u.chunk])
            off += u.chunk

    def apply_compile_plan(self, plan):
        """Install a schedule-compiler plan (compile/backend.py): kept groups are no longer
        released (their next fetch is their last until the plan changes), prefetches follow the
        compiled trigger table."""
        for fg in self.fgroups:
            for u in fg.units:
                u.keep = fg.idx in plan.get("keep", ()) and not u.persistent
        self.prefetch_plan = plan.get("prefetch")
        self.compile_plan = plan

    def zero_grad(self, set_to_none=True):
        for p in self.param_unit:
            p.grad = None

    # ---------------------------------------------------------------------- gathered-param access
    def gather_all(self, hold=True):
        """Gather every unit; with ``hold`` the module hooks do not release them until
        ``release_all`` (generation / evaluation phases of the hybrid engine)."""
        self.wait_params()
        for fg in self.fgroups:
            self._fetch(fg, wait=True)
        self._hold = bool(hold)

    def release_all(self):
        self._hold = False
        for fg in self.fgroups:
            self._release(fg)

    def empty_partition_cache(self):
        """Free every gathered non-persistent unit (engine.empty_partition_cache, reference
        stage3.py ``empty_partition_cache``): after evaluation or generation outside the training
        loop, the next forward gathers again."""
        self.wait_params()
        self._hold = False
        for units in self.units:
            for u in units:
                if not u.persistent and u.state != RELEASED:
                    self._release_unit(u)

    def gather_params(self, params):
        self.wait_params()
        owner = lambda p: self.param_unit.get(p) or self.frozen_unit.get(p)  # noqa: E731
        units = {id(owner(p)): owner(p) for p in params if owner(p) is not None}
        for u in units.values():
            if not u.persistent and u.state == RELEASED:
                self._launch_gather(u)
            if u.state == INFLIGHT:
                if u.event is not None:
                    torch.cuda.current_stream().wait_event(u.event)
                u.state = AVAILABLE
        return list(units.values())

    def commit_modified_units(self, units, src_rank=None, group=None):
        """After in-place edits of gathered params: optionally broadcast from `src_rank`, then
        refresh shards and fp32 masters from the full buffers."""
        self.wait_params()
        for u in units:
            if src_rank is not None:
                dist.broadcast(u.flat, src=src_rank, group=group)
            if getattr(u, "frozen", False):  # no master: the shard (or its int8 form) is the state
                if u.frozen_q:
                    from ...ops.quantizer import quantize
                    u.qshard = quantize(u.flat[u.lo:u.hi], self._qgroup(u), 8)
                elif not u.persistent:
                    u.shard.copy_(u.flat[u.lo:u.hi])
                continue
            if not u.persistent:
                u.shard.copy_(u.flat[u.lo:u.hi])
            if self.host_step is not None:
                self.host_step.write_master(self, u)
            else:
                u.master.copy_(u.shard.float())

    # ----------------------------------------------------------------------------- checkpointing
    def shuffle_exchange(self):
        self.wait_params()
        if self.se is not None:
            self.se.shuffle_exchange()

    def synchronization(self):
        self.wait_params()
        if self.se is not None and self.se.synchronization([u.shard for units in self.units for u in units]):
            self._refresh_persistent()

    def reset_rings(self, rings):
        if self.se is not None:
            self.se.reset_rings(rings)

    def unit_layout(self, name_of):
        return [[{"params": [name_of.get(p, "") for p in u.params], "shapes": u.shapes, "offsets": u.offsets,
                  "numel": u.numel, "padded": u.padded, "chunk": u.chunk} for u in units] for units in self.units]

    def state_dict(self):
        self.wait_params()
        self._host_materialize()
        return {
            "loss_scaler": self.loss_scaler.state_dict(),
            "dynamic_loss_scale": bool(getattr(self.loss_scaler, "dynamic", False)),
            "overflow": self.overflow,
            "clip_grad": self.clip_grad,
            "optimizer_state_dict": self.optimizer.state_dict(),
            "fp32_flat_groups": [m.data for m in self.master],
            "bit16_partitions": [[u.swap.read_copy(u) if u.swap is not None else u.shard for u in units]
                                 for units in self.units],
            "zero_stage": 3,
            "partition_count": self.S,
            "shuffle_exchange": self.se.state_dict() if self.se is not None else None,
            "ds_version": "sxe-0.1",
        }

    def load_state_dict(self, sd, load_optimizer_states=True, load_from_fp32_weights=True):
        self.wait_params()
        self.loss_scaler.load_state_dict(sd["loss_scaler"])
        self._host_materialize()
        if load_optimizer_states:
            self.optimizer.load_state_dict(sd["optimizer_state_dict"])
            for m in self.master:
                st = self.optimizer.state[m]
                for k, v in list(st.items()):
                    if isinstance(v, torch.Tensor) and v.numel() > 1:
                        st[k] = v.to(m.device)
        for m, saved in zip(self.master, sd["fp32_flat_groups"]):
            m.data.copy_(saved.to(m.device))
        for units in self.units:
            for u in units:
                u.shard_for_overwrite().copy_(u.master)
        if self.pswap is not None:
            self.pswap.flush()
        self._host_flush()
        self._refresh_persistent()
        if self.se is not None and sd.get("shuffle_exchange"):
            self.se.load_state_dict(sd["shuffle_exchange"])
