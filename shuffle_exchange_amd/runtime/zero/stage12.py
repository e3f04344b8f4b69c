"""ZeRO stage 1/2 optimizer with Shuffle-exchange hierarchical slices.

Parity: reference runtime/zero/stage_1_and_2.py:119 ``DeepSpeedZeroOptimizer`` (init :131-690,
grad hooks :1090-1102, bucketing :1114-1154, average_tensor :1242-1345, step :2058-2268,
state_dict :2472) including the fork's slice groups, inter-slice groups and the RR / shuffle / H-RR /
Gossip parameter synchronisation plus ``shuffle_exchange()``, ``synchronization()``,
``reset_rings()`` (stage_1_and_2.py:692-734).

Data flow per step on MI355X (slice of S ranks; with ``slice_count`` == DP world this is plain
ZeRO-1/2):
  backward: post-accumulate-grad hook copies each grad into its unit's staging buffer; when a unit
            is complete ONE reduce-scatter (slice group) lands the averaged chunk in the owner's
            fp32 accumulator -- on a dedicated HIP comm stream, overlapping the rest of backward.
            Stage 1 only reduces on the gradient-accumulation boundary micro-step; stage 2 every
            micro-step (and frees the full grads immediately).
  step:     device-side norm/clip/overflow -> one multi-tensor fused Adam launch that also writes the
            bit16 chunk -> inter-slice sync of the chunk (Shuffle-exchange) -> one in-place
            all-gather per unit inside the slice.
"""
import torch

from ... import comm as dist
from ...accelerator import get_accelerator
from ...utils.logging import log_dist
from .base import ZeroOptimizerBase
from .flat import FlatUnit, split_into_units
from .shuffle_exchange import ShuffleExchange, SliceTopology
from ..torch_autocast import split_by_comm_dtype, unit_comm_dtype


class ZeroStage12Optimizer(ZeroOptimizerBase):
    supports_overlapped_step = True  # zero/base.py _overlapped_update
    def __init__(self, init_optimizer, *, stage=2, loss_scaler, clip_grad=0.0, dp_ranks=None, dp_group=None,
                 reduce_bucket_size=500_000_000, communication_data_type=None, overlap_comm=True,
                 shuffle_exchange_cfg=None, method=None, slice_count=None, rings=None, shuffle_step=None,
                 mp_group=None, timers=None, average_master=False, host_step=None, fp32_accum=False):
        acc = get_accelerator()
        device = torch.device(acc.current_device_name())
        self.stage = stage
        dp_ranks = list(dp_ranks) if dp_ranks is not None else list(range(dist.get_world_size()))
        # ---- Shuffle-exchange topology ------------------------------------------------------------
        se = shuffle_exchange_cfg
        enabled = bool(se is not None and se.enabled) or any(v is not None for v in (method, slice_count))
        self.method = method or (se.method if se is not None else "RR")
        S = slice_count or (se.slice_count if (se is not None and se.enabled) else len(dp_ranks))
        if not enabled:
            S = len(dp_ranks)
        self.slice_count = S
        self.topo = SliceTopology(dp_ranks, S)
        self.shuffle_exchange_enabled = enabled and self.topo.num_slices > 1
        self.se = ShuffleExchange(self.topo, method=self.method,
                                  rings=rings or (se.rings if se is not None else 8),
                                  shuffle_step=shuffle_step or (se.shuffle_step if se is not None else 50),
                                  seed=se.seed if se is not None else 1234,
                                  gossip_p=se.gossip_p if se is not None else 1.0,
                                  average_master=average_master) if self.shuffle_exchange_enabled else None
        slice_group = self.topo.slice_group if self.topo.S > 1 else None
        world_group = dp_group if self.shuffle_exchange_enabled else None
        super().__init__(init_optimizer, loss_scaler, clip_grad, slice_group, overflow_group=world_group,
                         mp_group=mp_group, device=device)
        self.host_step = host_step
        # data_types.grad_accum_dtype == fp32 at stage 1 (reference BF16_Optimizer semantics,
        # runtime/bf16_optimizer.py:35, engine.py:1384-1386): micro-step gradients are summed in a
        # full-size fp32 buffer per unit instead of the bit16 .grad, and reduced (in fp32 unless
        # communication_data_type says otherwise) once at the accumulation boundary
        self.fp32_accum = bool(fp32_accum) and stage == 1
        self.comm_dtype = communication_data_type
        self.overlap_comm = overlap_comm
        self.comm_stream = acc.named_stream("zero_reduce") if (overlap_comm and acc.gpu) else None
        self.timers = timers
        self.micro_step_boundary = True
        self._hooks = []
        self.param_unit = {}
        self._moe_topos = {}
        # ---- flatten every param group into units -------------------------------------------------
        dtype = None
        for g, pg in enumerate(init_optimizer.param_groups):
            params = [p for p in pg["params"] if p.requires_grad]
            if not params:
                self.units.append([])
                continue
            dtype = params[0].dtype
            units = []
            # torch_autocast: runs of equal gradient-communication dtype get units of their own
            plists = [pl for run in split_by_comm_dtype(params)
                      for pl in split_into_units(run, max(1, int(reduce_bucket_size)))]
            for i, plist in enumerate(plists):
                gt = self._group_topo(pg)
                u = FlatUnit(plist, gt.S, gt.offset, dtype, device, name=f"g{g}u{i}", index=i)
                u.comm_dtype = unit_comm_dtype(plist)
                u.topo = gt
                u.moe = bool(pg.get("moe", False))
                if self.fp32_accum:
                    u.staging_dtype = torch.float32
                units.append(u)
                for p in plist:
                    self.param_unit[p] = u
            self.units.append(units)
        self.bit16_dtype = dtype
        if self._moe_topos:
            if self.shuffle_exchange_enabled:
                # Shuffle-exchange + MoE (reference stage_1_and_2.py:810-821): expert groups keep their
                # expert-data-parallel ZeRO partitioning across the slices (their gradient is the
                # global one, reduced over the expert-DP group and divided by the dense DP size), only
                # the dense groups are sliced and averaged between slices. The norm domain of the
                # dense part stays the slice; the expert sum of squares is summed world-wide.
                self._split_expert_norm = True
            else:
                # expert and dense partitions are disjoint across the whole DP group: one norm reduce
                self.partition_group = dp_group
        self._init_master()
        for units in self.units:  # fp32 accumulators start zeroed: every slot counts as written
            for u in units:
                u.acc_valid = [True] * len(u.params)
        self._register_hooks()
        self._module_units = None  # module -> units of its own params (set by attach_module)
        self._pending_events = {}  # unit -> HIP event of its post-step gather (consumed by forward)
        log_dist(f"ZeRO-{stage}: {sum(len(u) for u in self.units)} units, slice_count={S}, "
                 f"slices={self.topo.num_slices}, shuffle_exchange="
                 f"{self.method if self.shuffle_exchange_enabled else 'off'}", ranks=[0])

    def _group_topo(self, pg):
        if not pg.get("moe", False):
            return self.topo
        name = pg["name"]
        if name not in self._moe_topos:
            from ...parallel import groups
            ep = int(name.rsplit("_", 1)[-1]) if name.startswith("ep_size_") else None
            groups.create_expert_and_data_parallel(ep, name)
            edp = groups._Registry.expert[name][3]
            self._moe_topos[name] = SliceTopology(edp, len(edp))
        return self._moe_topos[name]

    # ------------------------------------------------------------------------------------- backward
    def _register_hooks(self):
        for p, u in self.param_unit.items():
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(u)))
            if (self.stage == 2 and u.topo.S > 1) or (u.topo.S == 1 and self._unit_scale(u) == 1.0):
                # weight-grad GEMMs (ops/linear.py) write into the fp32 accumulator (S == 1) or the
                # bf16 reduce-scatter staging slot (S > 1) directly
                p._sxe_grad_target = self._grad_target
                p._sxe_grad_done = self._grad_done
                if u.topo.S == 1:  # only this rank ever writes the accumulator: safe to write it late
                    p._sxe_grad_defer = self._grad_defer

    def _grad_target(self, p):
        u = self.param_unit[p]
        i = u.param_index[id(p)]
        o, n = u.offsets[i], u.numels[i]
        if u.topo.S == 1:  # the step's first write of the slot overwrites (GEMM beta = 0)
            return u.grad[o:o + n].view(p.shape), u.acc_valid[i]
        if u.staging is None:
            u.staging = torch.empty(u.padded, dtype=u.dtype, device=u.device)
            if u.padded > u.numel:
                u.staging[u.numel:].zero_()
        return u.staging[o:o + n].view(p.shape), u.filled[i]

    def _grad_done(self, p):
        u = self.param_unit[p]
        i = u.param_index[id(p)]
        if u.topo.S == 1:
            u.acc_valid[i] = True
        if not u.filled[i]:
            u.filled[i] = True
            u.pending -= 1
        if u.topo.S > 1 and u.pending == 0:
            self._reduce_unit(u)

    def _grad_defer(self, p):
        """May a weight-gradient producer hold this micro-step's contribution and write it at the
        accumulation boundary instead (moe/experts.py)? Yes before the boundary: a single-rank
        unit's accumulator is read by nothing until the step."""
        return not self.micro_step_boundary

    def grad_ready(self, p):
        """A gradient delivered outside autograd's AccumulateGrad (the FX graph compiler's in-graph
        reduce nodes, compile/fx_backend.py): ``p.grad`` is set; run the per-parameter hook."""
        u = self.param_unit.get(p)
        if u is not None:
            self._make_hook(u)(p)

    def _make_hook(self, unit):
        def hook(p):
            if p.grad is None or getattr(p, "_sxe_grad_partial", False):
                return  # partial tile gradient: keep summing in .grad until the last tile
            if not self.micro_step_boundary and self.stage == 1:
                # ZeRO-1 keeps accumulating full grads until the boundary: in the bit16 .grad
                # (autograd's own accumulation), or with fp32_accum in the unit's fp32 buffer
                if self.fp32_accum:
                    self._accumulate_fp32(unit, p)
                return
            if unit.topo.S == 1:
                i = unit.param_index[id(p)]
                self._acc_write(unit, i, p.grad, self._unit_scale(unit))
                unit.filled[i] = True
                p.grad = None
                return
            done = unit.stage_grad(p, p.grad)
            p.grad = None
            if done:
                self._reduce_unit(unit)
        return hook

    def _acc_write(self, u, i, src, alpha):
        """Add ``alpha * src`` into slot i of a single-rank unit's fp32 accumulator -- or overwrite
        it, when the slot is stale (its first write of the step: zero_grad_buffers)."""
        o, n = u.offsets[i], u.numels[i]
        dst = u.grad[o:o + n]
        src = src.reshape(-1)
        if u.acc_valid[i]:
            dst.add_(src, alpha=alpha)
        else:
            if src.dtype == dst.dtype:
                torch.mul(src, alpha, out=dst)
            else:
                dst.copy_(src)
                if alpha != 1.0:
                    dst.mul_(alpha)
            u.acc_valid[i] = True

    def _accumulate_fp32(self, unit, p):
        if unit.topo.S == 1:
            self._acc_write(unit, unit.param_index[id(p)], p.grad, self._unit_scale(unit))
        else:
            unit.stage_grad(p, p.grad)  # fp32 staging (staging_dtype), no reduce before the boundary
        p.grad = None

    def set_gradient_accumulation_boundary(self, flag):
        self.micro_step_boundary = bool(flag)

    def backward_prologue(self):
        self.drain_step()  # the update read the fp32 gradient accumulators the backward rewrites
        for units in self.units:
            for u in units:
                u.begin_backward()

    def _unit_scale(self, u):
        """Gradient averaging factor of a unit. Dense: the mean over its slice (x sp for sequence
        parallelism). Expert units are SUMMED over their expert-data-parallel group and divided by
        the dense data-parallel size, so the expert gradients do not depend on ep_size (reference
        stage_1_and_2.py:1316 divides the whole bucket by the dp group size; engine.py:2713-2716) --
        an EDP group of one rank (ep == dp) still averages over the dp ranks whose tokens it saw."""
        return self.sp_scale / (self.topo.W if getattr(u, "moe", False) else u.topo.S)

    def _reduce_unit(self, u):
        st = u.staging
        u.staging = None
        u.carry = False
        cur = torch.cuda.current_stream() if st.is_cuda else None
        stream = self.comm_stream
        if stream is not None:
            stream.wait_stream(cur)
        with get_accelerator().stream(stream):
            want = u.comm_dtype or self.comm_dtype
            send = st if (want is None or st.dtype == want) else st.to(want)
            out = torch.empty(u.chunk, dtype=send.dtype, device=send.device)
            dist.reduce_scatter_tensor(out, send, group=u.topo.slice_group)
            u.grad.add_(out, alpha=self._unit_scale(u))
            if stream is not None:
                st.record_stream(stream)
                send.record_stream(stream)
                out.record_stream(stream)

    def reduce_gradients(self, pipeline_parallel=False):
        """Backward epilogue: reduce units whose params did not all produce grads (unused params)
        and, for ZeRO-1 at the boundary, everything still pending."""
        if self.micro_step_boundary:
            from ...moe.experts import flush_deferred_wgrad
            from ...ops.mlp import flush_stashed_wgrad
            for p in self.param_unit:
                if p.__dict__.get("_sxe_wstash"):  # deferred weight grads no boundary backward consumed
                    flush_deferred_wgrad(p)
                if p.__dict__.get("_sxe_bstash") is not None:  # held bf16 weight grads (ops/mlp.py)
                    flush_stashed_wgrad(p)
        if self.stage == 1 and not self.micro_step_boundary:
            if self.fp32_accum:  # the fp32 staging sums carry into the next micro-step
                for units in self.units:
                    for u in units:
                        for i, p in enumerate(u.params):
                            if p.grad is not None:  # no hook fired (e.g. grads set outside autograd)
                                self._accumulate_fp32(u, p)
                        if u.staging is not None:
                            if not u.carry and u.pending > 0:
                                # slots of params without a gradient in this first micro-step
                                # are uninitialised (torch.empty staging): zero them before the
                                # later micro-steps add into them
                                u.fill_missing()
                            u.carry = True
            return
        for units in self.units:
            for u in units:
                if u.topo.S == 1:
                    # grads still held in .grad (accumulated before the boundary, e.g. pipeline
                    # micro-batches) go straight into the fp32 accumulator
                    for i, p in enumerate(u.params):
                        if p.grad is not None:
                            self._acc_write(u, i, p.grad, self._unit_scale(u))
                            p.grad = None
                    continue
                if u.pending > 0:
                    # params whose grads exist but whose hook did not fire (e.g. stage 1 grads
                    # accumulated before a boundary without a new backward contribution)
                    for i, p in enumerate(u.params):
                        if not u.filled[i] and p.grad is not None:
                            u.stage_grad(p, p.grad)
                            p.grad = None
                    if u.pending > 0:
                        u.fill_missing()
                    self._reduce_unit(u)

    def _wait_comm(self):
        self._drain_pending()
        if self.comm_stream is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)

    # ----------------------------------------------------------------------------------------- step
    def zero_grad_buffers(self):
        """Single-rank units (their accumulator is only ever written by this rank's backward) are
        marked stale instead of zeroed -- an 11.9 B-parameter Mixtral step spent 7 ms in that
        memset: each slot's first write of the next step overwrites and the slots no gradient
        reached are zeroed right before the update (_zero_stale). Units that reduce-scatter into
        their accumulator (add_) are zeroed as before."""
        for p in self.param_unit:
            p.__dict__.pop("_sxe_bstash", None)  # a partial accumulation goes with the rest
        multi = [u for units in self.units for u in units if u.topo.S > 1]
        if len(multi) == sum(len(us) for us in self.units):
            return super().zero_grad_buffers()
        for units in self.units:
            for u in units:
                if u.topo.S == 1:
                    u.acc_valid = [False] * len(u.params)
        if multi:
            if self.__dict__.get("_step_inflight"):
                from ...accelerator import get_accelerator
                with get_accelerator().stream(self._step_stream):
                    for u in multi:
                        u.grad.zero_()
            else:
                for u in multi:
                    u.grad.zero_()

    def _zero_stale(self):
        if self.host_step is not None:
            self.host_step.wait_grad_mirror()  # the async host update's D2H may still read u.grad
        for units in self.units:
            for u in units:
                if u.topo.S == 1 and not all(u.acc_valid):
                    for i, ok in enumerate(u.acc_valid):
                        if not ok:
                            o, n = u.offsets[i], u.numels[i]
                            u.grad[o:o + n].zero_()
                    u.acc_valid = [True] * len(u.params)

    def step(self, closure=None, lr_kwargs=None):
        self._wait_comm()
        self._zero_stale()
        if self.se is not None and self.method == "Gossip":
            self.se.pre_step([u.shard for u in self._dense_units()])
        coef, skip = self._grad_norm_and_flags()
        if getattr(self.loss_scaler, "dynamic", False):
            if self._handle_overflow_host():
                self.zero_grad_buffers()
                return
        self._fused_update(coef, skip)
        self.zero_grad_buffers()
        self._post_step_exchange()
        self.global_step += 1

    def attach_module(self, module):
        """Let the next forward overlap the post-step parameter exchange: every module that owns
        parameters gets a pre-forward hook that waits (on the device, no host sync) for the
        events of its own units only, so layer 0 computes while later units still gather."""
        mu = {}
        for m in module.modules():
            us = []
            for p in m.parameters(recurse=False):
                u = self.param_unit.get(p)
                if u is not None and u not in us:
                    us.append(u)
            if us:
                mu[m] = us
                self._hooks.append(m.register_forward_pre_hook(self._make_wait_hook(us)))
        self._module_units = mu

    def _make_wait_hook(self, units):
        def pre(mod, args):
            if not self._pending_events:
                return
            cur = torch.cuda.current_stream()
            for u in units:
                ev = self._pending_events.pop(u, None)
                if ev is not None:
                    cur.wait_event(ev)
        return pre

    def _post_step_exchange(self):
        """Inter-slice synchronisation (Shuffle-exchange) and the in-slice all-gather, unit by unit
        on the comm stream: the Shuffle-exchange all-reduce of unit k+1 overlaps nothing on the
        comm stream but the all-gather of unit k is already done, and the compute stream is free
        to start the next forward (it waits per unit via ``attach_module``'s hooks)."""
        units = [u for us in self.units for u in us]
        masters = self._device_masters()
        stream = self.comm_stream if self._module_units is not None else None
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream())
        evs = self.__dict__.get("_step_events") or {}
        if evs and (self.se is not None or stream is None):
            self.drain_step()  # chunks needed all at once (inter-slice sync) / no per-unit consumer
            if stream is not None:
                stream.wait_stream(torch.cuda.current_stream())
            evs = {}
        with get_accelerator().stream(stream):
            if self.se is not None:
                # one packed inter-slice collective per step for all dense chunks (Gossip: one plan);
                # expert chunks are already identical across their expert-DP group
                dense = self._dense_units()
                if masters is not None:
                    masters = [u.master for u in dense]
                self.se.sync([u.shard for u in dense], masters)
            for i, u in enumerate(units):
                ev = evs.pop(u, None)  # this unit's overlapped update (zero/base.py)
                if ev is not None and u.topo.S > 1:
                    stream.wait_event(ev)
                elif ev is not None:  # nothing to gather: the forward hook of its module waits
                    self._pending_events[u] = ev
                    continue
                if u.topo.S > 1:
                    dist.all_gather_into_tensor(u.flat, u.shard, group=u.topo.slice_group)
                if stream is not None:
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    self._pending_events[u] = ev
        # units no forward hook consumed are waited for by the next step / checkpoint at the latest

    def wait_params(self):
        """Make the compute stream wait for every in-flight post-step parameter exchange."""
        self._drain_pending()

    def _drain_pending(self):
        self.drain_step()
        if self._pending_events:
            cur = torch.cuda.current_stream()
            for ev in self._pending_events.values():
                cur.wait_event(ev)
            self._pending_events.clear()

    def _allgather_params(self):
        self._drain_pending()
        for units in self.units:
            for u in units:
                if u.topo.S > 1:
                    dist.all_gather_into_tensor(u.flat, u.shard, group=u.topo.slice_group)

    def zero_grad(self, set_to_none=True):
        for p in self.param_unit:
            p.grad = None

    # ---------------------------------------------------------------------- Shuffle-exchange hooks
    def _dense_units(self):
        return [u for units in self.units for u in units if not getattr(u, "moe", False)]

    def shuffle_exchange(self):
        if self.se is not None:
            self.se.shuffle_exchange()

    def synchronization(self):
        if self.se is not None and self.se.synchronization([u.shard for u in self._dense_units()]):
            self._allgather_params()

    def reset_rings(self, rings):
        if self.se is not None:
            self.se.reset_rings(rings)

    # ------------------------------------------------------------------------------- checkpointing
    def unit_layout(self, name_of):
        return [[{"params": [name_of.get(p, "") for p in u.params], "shapes": u.shapes, "offsets": u.offsets,
                  "numel": u.numel, "padded": u.padded, "chunk": u.chunk} for u in units] for units in self.units]

    def param_slice_mappings(self, name_of):
        """Per param group {param name: {"numel", "start"}}: the fragment of each parameter held
        in this rank's flat fp32 partition (reference stage_1_and_2.py:2510 ``param_slice_mappings``
        of ``fragment_address(numel, start)``), plus ``param_start``, the fragment's first element
        inside the parameter (the units are not padded per parameter, so a fragment can start
        mid-parameter on any rank)."""
        out = []
        for units in self.units:
            m, base = {}, 0
            for u in units:
                for i, p in enumerate(u.params):
                    r = u.param_range_in_shard(i)
                    if r is not None:
                        plo, phi, slo = r
                        m[name_of.get(p, f"param_{id(p)}")] = {"numel": phi - plo, "start": base + slo,
                                                               "param_start": plo}
                base += u.chunk
            out.append(m)
        return out

    def state_dict(self):
        self.wait_params()
        self._host_materialize()
        return {
            "loss_scaler": self.loss_scaler.state_dict(),
            "dynamic_loss_scale": bool(getattr(self.loss_scaler, "dynamic", False)),
            "overflow": self.overflow,
            "clip_grad": self.clip_grad,
            "base_optimizer_state": self.optimizer.state_dict(),
            "single_partition_of_fp32_groups": [m.data for m in self.master],
            "zero_stage": self.stage,
            "group_paddings": [sum(u.padded - u.numel for u in units) for units in self.units],
            "partition_count": [self.topo.S for _ in self.units],
            "shuffle_exchange": self.se.state_dict() if self.se is not None else None,
            "slice_count": self.topo.S,
            "ds_version": "sxe-0.1",
        }

    def load_state_dict(self, sd, load_optimizer_states=True, load_from_fp32_weights=True):
        self.wait_params()
        self.loss_scaler.load_state_dict(sd["loss_scaler"])
        self.clip_grad = sd.get("clip_grad", self.clip_grad)
        self._host_materialize()
        if load_optimizer_states:
            saved = sd["base_optimizer_state"]
            self.optimizer.load_state_dict(saved)
            # load_state_dict re-binds state to our master params; make sure tensors are on device
            for m in self.master:
                st = self.optimizer.state[m]
                for k, v in list(st.items()):
                    if isinstance(v, torch.Tensor) and v.numel() > 1:
                        st[k] = v.to(m.device)
        if load_from_fp32_weights:
            for m, saved in zip(self.master, sd["single_partition_of_fp32_groups"]):
                m.data.copy_(saved.to(m.device))
            for units in self.units:
                for u in units:
                    u.shard.copy_(u.master)
            self._allgather_params()
        self._host_flush()
        if self.se is not None and sd.get("shuffle_exchange"):
            self.se.load_state_dict(sd["shuffle_exchange"])
