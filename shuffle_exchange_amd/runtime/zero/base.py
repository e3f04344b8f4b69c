"""Shared machinery of the ZeRO optimizers: fp32 master chunks, fused optimizer step, device-side
clipping/overflow, state dicts.

Parity: the step half of reference runtime/zero/stage_1_and_2.py:2058-2268 (norm :1941, clip
:2018-2032, optimizer step :2039-2053, fp32->bit16 copy :2174-2176) and stage3.py:2112-2174.
MI355X-first: the whole step is asynchronous on the device -- the gradient norm, the
non-finite check and the clip coefficient stay in device scalars that the fused HIP optimizer
kernel reads (``scale_t``/``skip_t``), so bf16 training never synchronises the host in ``step()``
(the reference calls ``.item()`` on the overflow flag every step, stage_1_and_2.py:2073,2342).
"""
import torch

from ... import comm as dist
from ...ops import optim as fused
from ...utils.logging import log_dist


def _kind(opt):
    from torch.optim import Adam, AdamW, Adagrad
    if isinstance(opt, fused.FusedAdam):
        return "adam", opt.adam_w_mode
    if isinstance(opt, AdamW):
        return "adam", True
    if isinstance(opt, Adam):
        return "adam", False
    if isinstance(opt, fused.FusedLion):
        return "lion", None
    if isinstance(opt, (fused.FusedAdagrad, Adagrad)):
        return "adagrad", None
    if isinstance(opt, fused.FusedLamb):
        return "lamb", None
    return "generic", None


class ZeroOptimizerBase:
    """Holds, per parameter group ``g``: ``units[g]`` (FlatUnit list), ``master[g]`` (fp32 chunk
    concatenation), ``grads[g]`` (fp32 chunk gradient accumulator)."""

    def __init__(self, init_optimizer, loss_scaler, clip_grad, partition_group, overflow_group=None,
                 mp_group=None, device=None):
        self.optimizer = init_optimizer
        self.loss_scaler = loss_scaler
        self.clip_grad = float(clip_grad or 0.0)
        self.partition_group = partition_group
        self.overflow_group = overflow_group
        self.mp_group = mp_group
        self.device = device
        self.kind, self.adamw = _kind(init_optimizer)
        self.units = []
        self.master = []
        self.grads = []
        self.overflow = False
        self._last_norm = None
        self._skip_t = None
        self.global_step = 0
        # Ulysses SP: ranks of one SP group hold different tokens of the same sequences, so their
        # gradients are summed while data-parallel replicas are averaged: reduce-scatter results are
        # scaled by sp / |DP x SP| (reference divides by dp/sp, stage_1_and_2.py:1314)
        self.sp_scale = 1.0
        # ZeRO-Offload / ZeRO-Infinity (runtime/zero/offload.py): masters + optimizer state on the
        # host or NVMe, update by the C++ CPU kernels; None = everything on the GPU
        self.host_step = None

    def destroy(self):
        """Remove every hook this optimizer installed on parameters / modules and finish in-flight
        exchanges (engine.destroy, reference engine.py:521-530)."""
        if hasattr(self, "wait_params"):
            self.wait_params()
        for h in getattr(self, "_hooks", []):
            h.remove()
        self._hooks = []
        self._module_hooks = []
        for units in self.units:
            for u in units:
                for p in u.params:
                    for a in ("_sxe_grad_target", "_sxe_grad_done"):
                        if hasattr(p, a):
                            delattr(p, a)

    # --------------------------------------------------------------------------------------------
    def _init_master(self):
        """Create fp32 masters/grad accumulators and re-point the wrapped optimizer at them."""
        for g, units in enumerate(self.units):  # lp -> hp linkage for utils/tensor_fragment.py
            for u in units:
                for i, p in enumerate(u.params):
                    p._sxe_zero = (self, g, u, i)
        G = len(self.units)
        self.master, self.grads = [None] * G, [None] * G
        host = self.host_step.host_groups(self) if self.host_step is not None else set()
        for g, units in enumerate(self.units):
            if g in host:
                continue  # masters / state on the host tier (offload.py)
            total = sum(u.chunk for u in units)
            m = torch.empty(total, dtype=torch.float32, device=self.device)
            gr = torch.zeros(total, dtype=torch.float32, device=self.device)
            off = 0
            for u in units:
                u.master = m[off:off + u.chunk]
                u.grad = gr[off:off + u.chunk]
                u.master.copy_(u.shard.float())
                off += u.chunk
            m = torch.nn.Parameter(m, requires_grad=False)
            self.master[g] = m
            self.grads[g] = gr
            self.optimizer.param_groups[g]["params"] = [m]
        if self.host_step is not None:
            return self.host_step.init_master(self)  # also initialises the state of every group
        self.optimizer.state.clear()
        self._init_state()

    def _init_state(self):
        for g, m in enumerate(self.master):
            st = self.optimizer.state[m]
            if self.kind in ("adam", "lamb"):
                st["step"] = 0
                st["exp_avg"] = torch.zeros_like(m.data)
                st["exp_avg_sq"] = torch.zeros_like(m.data)
            elif self.kind == "lion":
                st["exp_avg"] = torch.zeros_like(m.data)
            elif self.kind == "adagrad":
                st["sum"] = torch.zeros_like(m.data)
                st["step"] = 0

    # --------------------------------------------------------------------------------------------
    def _norm_domains(self):
        """Step-metadata layout, built once (collectively) on the first step.

        The gradient norm of a rank is summed over its *norm domain*: the ranks holding different
        pieces of the same model replica's gradients -- the connected closure of its partition
        group (ZeRO chunks, or a Shuffle-exchange slice) and its model-parallel group (TP x PP).
        The non-finite flag is agreed world-wide (the fork's world overflow check, reference
        stage_1_and_2.py:2071-2073). Both travel in ONE all-reduce of a [D + 1] fp32 vector over
        the world: slot ``domain`` carries this rank's sum of squares, slot D the non-finite count
        (reference: a norm all-reduce per group plus a separate overflow all-reduce)."""
        if getattr(self, "_meta", None) is not None:
            return self._meta
        W = dist.get_world_size()
        if W == 1:
            self._meta = (0, 1)
            return self._meta
        part = dist.group_ranks(self.partition_group) if self.partition_group is not None else [dist.get_rank()]
        mp = dist.group_ranks(self.mp_group) if self.mp_group is not None else [dist.get_rank()]
        extra = getattr(self, "extra_norm_group", None)
        mp = list(mp) + (dist.group_ranks(extra) if extra is not None else [])
        objs = [None] * W
        import torch.distributed as tdist
        tdist.all_gather_object(objs, (tuple(part), tuple(mp)))
        parent = list(range(W))

        def find(a):
            while parent[a] != a:
                parent[a] = parent[parent[a]]
                a = parent[a]
            return a
        for r, (pr, mr) in enumerate(objs):
            for q in list(pr) + list(mr):
                ra, rb = find(r), find(q)
                if ra != rb:
                    parent[max(ra, rb)] = min(ra, rb)
        roots = sorted({find(r) for r in range(W)})
        self._meta = (roots.index(find(dist.get_rank())), len(roots))
        return self._meta

    def _grad_norm_and_flags(self):
        """Device-side: global grad norm (unscaled), the clip/unscale coefficient and the skip
        (non-finite) flag, with ONE small all-reduce for all step metadata. No host sync."""
        # Shuffle-exchange + MoE (stage12): expert groups are partitioned over expert-DP groups that
        # span the slices, so their sum of squares is summed world-wide in a slot of its own
        split = bool(getattr(self, "_split_expert_norm", False))
        sq = sq_e = None
        for g, gr in enumerate(self.grads):
            s = fused.sumsq(gr)
            pg = self.optimizer.param_groups[g] if g < len(self.optimizer.param_groups) else {}
            w = pg.get("norm_weight", 1.0)
            if w != 1.0:
                s = s * w
            if split and pg.get("moe", False):
                sq_e = s if sq_e is None else sq_e + s
            else:
                sq = s if sq is None else sq + s
        sq = sq.reshape(1).float() if sq is not None else torch.zeros(1, dtype=torch.float32, device=self.device)
        domain, D = self._norm_domains()
        if D > 1 or dist.get_world_size() > 1:
            E = 1 if split else 0
            meta = torch.zeros(D + E + 1, dtype=torch.float32, device=sq.device)
            meta[domain:domain + 1] = torch.nan_to_num(sq, nan=0.0, posinf=0.0)
            bad = (~torch.isfinite(sq)).float()
            if split:
                sq_e = sq_e.reshape(1).float() if sq_e is not None else torch.zeros_like(sq)
                meta[D:D + 1] = torch.nan_to_num(sq_e, nan=0.0, posinf=0.0)
                bad = bad + (~torch.isfinite(sq_e)).float()
            meta[D + E:] = bad
            dist.all_reduce(meta, group=None, log_name="step_meta")
            tot = meta[domain:domain + 1] + (meta[D:D + 1] if split else 0.0)
            # a non-finite gradient anywhere in the world -> inf norm -> every rank skips the step
            sq = torch.where(meta[D + E:] > 0, torch.full_like(sq, float("inf")), tot)
        ls = float(self.loss_scaler.loss_scale)
        norm = sq.sqrt() / ls
        skip = (~torch.isfinite(norm)).float()
        coef = torch.full((1,), 1.0 / ls, dtype=torch.float32, device=norm.device)
        if self.clip_grad > 0:
            clip = torch.clamp(self.clip_grad / (torch.nan_to_num(norm, nan=0.0, posinf=0.0) + 1e-6), max=1.0)
            coef = coef * clip
        self._last_norm = norm
        self._skip_t = skip
        return coef, skip

    def _fused_update(self, coef, skip):
        """One optimizer step over every unit chunk; writes the bit16 chunks in the same pass."""
        host = set()
        if self.host_step is not None:
            self.host_step.update(self, coef, skip)
            host = self.host_step.groups
            if len(host) == len(self.units):
                return
        for g, units in enumerate(self.units):
            if g in host:
                continue  # Twin-Flow: this group was stepped on the host
            pg = self.optimizer.param_groups[g]
            m = self.master[g]
            st = self.optimizer.state[m]
            if self.kind == "adam":
                st["step"] = int(st.get("step", 0)) + 1
                b1, b2 = pg["betas"]
                if m.is_cuda:
                    offs = self._unit_offsets(g)

                    def adam(us):
                        idx = [units.index(u) for u in us] if us is not units else range(len(units))
                        torch.ops.sxe.multi_tensor_adam_(
                            [units[j].master for j in idx], [units[j].grad for j in idx],
                            [st["exp_avg"][offs[j]:offs[j] + units[j].chunk] for j in idx],
                            [st["exp_avg_sq"][offs[j]:offs[j] + units[j].chunk] for j in idx],
                            [units[j].shard for j in idx], coef, skip, float(pg["lr"]), float(b1), float(b2),
                            float(pg["eps"]), float(pg["weight_decay"]), int(st["step"]), bool(self.adamw),
                            bool(pg.get("bias_correction", True)), 1.0)
                    if self._overlap_step_ok(units):
                        self._overlapped_update(units, adam, coef, skip)
                    else:
                        adam(units)
                else:
                    offs = self._unit_offsets(g)
                    for u, o in zip(units, offs):
                        fused.adam_flat_(u.master, u.grad, st["exp_avg"][o:o + u.chunk],
                                         st["exp_avg_sq"][o:o + u.chunk], u.shard, lr=pg["lr"], beta1=b1, beta2=b2,
                                         eps=pg["eps"], weight_decay=pg["weight_decay"], step=st["step"],
                                         adamw=self.adamw, bias_correction=pg.get("bias_correction", True),
                                         scale_t=coef, skip_t=skip)
            elif self.kind == "lion":
                b1, b2 = pg["betas"]
                for u, o in zip(units, self._unit_offsets(g)):
                    fused.lion_flat_(u.master, u.grad, st["exp_avg"][o:o + u.chunk], u.shard, lr=pg["lr"], beta1=b1,
                                     beta2=b2, weight_decay=pg["weight_decay"], scale_t=coef, skip_t=skip)
            elif self.kind == "adagrad":
                st["step"] = int(st.get("step", 0)) + 1
                for u, o in zip(units, self._unit_offsets(g)):
                    fused.adagrad_flat_(u.master, u.grad, st["sum"][o:o + u.chunk], u.shard, lr=pg["lr"],
                                        eps=pg.get("eps", 1e-10), weight_decay=pg.get("weight_decay", 0.0),
                                        scale_t=coef, skip_t=skip)
            elif self.kind == "lamb":
                st["step"] = int(st.get("step", 0)) + 1
                b1, b2 = pg["betas"]
                table, nseg = self._lamb_segments(g)
                lp = units[0].shard if len(units) == 1 else None
                fused.lamb_flat_(m.data, self.grads[g], st["exp_avg"], st["exp_avg_sq"], lp, table, nseg, lr=pg["lr"],
                                 beta1=b1, beta2=b2, eps=pg["eps"], weight_decay=pg["weight_decay"], step=st["step"],
                                 bias_correction=pg.get("bias_correction", True), min_coeff=pg.get("min_coeff", 0.01),
                                 max_coeff=pg.get("max_coeff", 10.0), scale_t=coef, skip_t=skip,
                                 norm_group=self.partition_group if any(u.S > 1 for u in units) else None)
                if lp is None:  # several units: refresh each unit's bit16 shard from its master chunk
                    for u in units:
                        u.shard.copy_(u.master)
        if self.kind == "generic":
            # any torch.optim optimizer: fp32 grads -> .grad of the master, step, copy back.
            # (host-synchronising on skip; the fused kinds above never do)
            if float(skip.reshape(-1)[0]) != 0.0:
                return
            for g, m in enumerate(self.master):
                m.grad = self.grads[g] * coef
            self.optimizer.step()
            for g, units in enumerate(self.units):
                self.master[g].grad = None
                for u in units:
                    u.shard.copy_(u.master)

    # ------------------------------------------------------------ overlapped device update
    # SXE_STEP_OVERLAP=1 (opt-in, ZeRO-1/2/3 with fused Adam on the GPU): the update runs on a side
    # stream as one launch per unit in the order the next forward needs the units, and every
    # consumer waits for exactly its own units' event (forward pre-hooks, the post-step gathers),
    # so the HBM-bound update of the later units can run beside the MFMA-bound forward of the
    # earlier ones. Same kernel, same math per element: bit-identical results. Off by default: on
    # one MI355X the hipBLASLt GEMMs leave no room for concurrent update workgroups -- 25,363 vs
    # 25,387 tokens/s (Llama-3-8B) and 24,962 vs 25,020 (Mixtral), profiles/r05/step_overlap_*.log.
    def _overlap_step_ok(self, units):
        if not getattr(self, "supports_overlapped_step", False) or not units or not units[0].master.is_cuda:
            return False
        if not hasattr(self, "_overlap_on"):
            import os
            self._overlap_on = os.environ.get("SXE_STEP_OVERLAP", "0") == "1"
        return self._overlap_on

    def _overlapped_update(self, units, adam, coef, skip):
        from ...accelerator import get_accelerator
        acc = get_accelerator()
        if getattr(self, "_step_stream", None) is None:
            self._step_stream = acc.named_stream("zero_step")
            self._step_events = {}
        ss = self._step_stream
        ss.wait_stream(torch.cuda.current_stream())
        self._step_inflight = True
        rank = {id(u): r for r, u in enumerate(self.step_unit_order())}
        order = sorted(units, key=lambda u: rank.get(id(u), len(rank)))
        with acc.stream(ss):
            for u in order:
                adam([u])
                ev = torch.cuda.Event()
                ev.record(ss)
                self._step_events[u] = ev
        coef.record_stream(ss)
        skip.record_stream(ss)

    def step_unit_order(self):
        """Units in the order the next forward consumes them (ZeRO-3 overrides with its trace)."""
        return [u for us in self.units for u in us]

    def wait_step_unit(self, u, stream=None):
        """Make ``stream`` (default: the current one) wait until unit ``u``'s update has run."""
        ev = self.__dict__.get("_step_events", {}).pop(u, None) if stream is None else \
            self.__dict__.get("_step_events", {}).get(u)
        if ev is not None:
            (stream or torch.cuda.current_stream()).wait_event(ev)

    def drain_step(self):
        """The current stream waits for every pending overlapped update (and the accumulator
        zeroing queued behind it), whether or not its per-unit events were consumed."""
        if self.__dict__.get("_step_inflight"):
            torch.cuda.current_stream().wait_stream(self._step_stream)
            self._step_events.clear()
            self._step_inflight = False

    def _lamb_segments(self, g):
        """Per-parameter segments of group g's flat master on this rank (cached): LAMB's trust
        ratio is per ORIGINAL parameter, and a parameter split across the partition has its
        fragments' norms summed over the partition group."""
        cache = self.__dict__.setdefault("_lamb_tables", {})
        if g not in cache:
            segs, gi, base = [], 0, 0
            for u in self.units[g]:
                for i in range(len(u.params)):
                    rng = u.param_range_in_shard(i)
                    if rng is not None:
                        plo, phi, slo = rng
                        segs.append((gi, base + slo, phi - plo))
                    gi += 1
                base += u.chunk
            cache[g] = (fused.lamb_block_table(segs, self.master[g].device), gi)
        return cache[g]

    def _unit_offsets(self, g):
        offs, o = [], 0
        for u in self.units[g]:
            offs.append(o)
            o += u.chunk
        return offs

    def _device_masters(self):
        """Masters for collective averaging (shuffle-exchange average_master); None if offloaded."""
        if self.host_step is not None:
            return None
        return [u.master for units in self.units for u in units]

    def _host_materialize(self):
        if self.host_step is not None:
            self.host_step.materialize(self)

    def _host_flush(self):
        if self.host_step is not None and self.host_step.device == "nvme":
            self.host_step.flush(self)

    # ----------------------------------------------------------------------- offload_states API
    def _rebind_views(self):
        for g, units in enumerate(self.units):
            off = 0
            for u in units:
                if self.master[g].numel():
                    u.master = self.master[g].data[off:off + u.chunk]
                u.grad = self.grads[g][off:off + u.chunk]
                off += u.chunk

    def offload_states(self, include=None, device="cpu", pin_memory=True, non_blocking=False):
        """Move optimizer states / fp32 masters / grad accumulators (and ZeRO-3 bit16 shards) to the
        host to free HBM between phases (reference runtime/zero/offload_states.py:17-71)."""
        if hasattr(self, "wait_params"):
            self.wait_params()
        inc = set(include or ["optim_states", "hp_params", "lp_grads", "lp_params"])
        pin = pin_memory and torch.cuda.is_available()

        # pinned host buffers are kept across offload/reload cycles (per-step offloading, e.g.
        # engine.compile's offload_opt_states, must not pay a pinned allocation every step)
        cache = self.__dict__.setdefault("_pinned_host", {})

        def mv(t, *slot):
            if t is None or not torch.is_tensor(t) or t.device.type == "cpu":
                return t
            key = (slot, tuple(t.shape), t.dtype)
            h = cache.get(key)
            if h is None:
                if pin:
                    from .offload import pinned_empty
                    h = pinned_empty(t.numel(), t.dtype).view(t.shape)
                else:
                    h = torch.empty(t.shape, dtype=t.dtype)
                cache[key] = h
            h.copy_(t, non_blocking=non_blocking)
            return h

        self._offloaded = getattr(self, "_offloaded", {})
        if "hp_params" in inc:
            for gi, m in enumerate(self.master):
                self._offloaded.setdefault("dev", m.device)
                m.data = mv(m.data, "hp", gi)
        if "lp_grads" in inc:
            self.grads = [mv(g, "grad", gi) for gi, g in enumerate(self.grads)]
        if "optim_states" in inc:
            for gi, m in enumerate(self.master):
                st = self.optimizer.state[m]
                for k, v in list(st.items()):
                    if torch.is_tensor(v) and v.numel() > 1:
                        st[k] = mv(v, "opt", gi, k)
        if "lp_params" in inc and getattr(self, "fgroups", None) is not None:
            for gi, units in enumerate(self.units):
                for ui, u in enumerate(units):
                    if not u.persistent:
                        u.shard = mv(u.shard, "lp", gi, ui)
        self._rebind_views()
        self._offloaded["include"] = inc
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def reload_states(self, non_blocking=False):
        if hasattr(self, "wait_params"):
            self.wait_params()
        dev = self.device
        inc = getattr(self, "_offloaded", {}).get("include", set())

        def back(t):
            return t.to(dev, non_blocking=non_blocking) if torch.is_tensor(t) and t.device != dev else t

        host = self.host_step.groups if self.host_step is not None else set()
        if "hp_params" in inc:
            for g, m in enumerate(self.master):
                if g not in host:
                    m.data = back(m.data)
        if "lp_grads" in inc:
            self.grads = [back(g) for g in self.grads]
        if "optim_states" in inc:
            for g, m in enumerate(self.master):
                if g in host:
                    continue
                st = self.optimizer.state[m]
                for k, v in list(st.items()):
                    if torch.is_tensor(v) and v.numel() > 1:
                        st[k] = back(v)
        if "lp_params" in inc and getattr(self, "fgroups", None) is not None:
            for units in self.units:
                for u in units:
                    if not u.persistent and not getattr(self, "offload_param", False):
                        u.shard = back(u.shard)
        self._rebind_views()
        self._offloaded = {}

    def zero_grad_buffers(self):
        if self.__dict__.get("_step_inflight"):
            # the overlapped update still reads the accumulators: zero them behind it, on its stream
            from ...accelerator import get_accelerator
            with get_accelerator().stream(self._step_stream):
                for gr in self.grads:
                    gr.zero_()
            return
        for gr in self.grads:
            gr.zero_()

    # --------------------------------------------------------------------------------------------
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    @property
    def loss_scale(self):
        return self.loss_scaler.loss_scale

    @property
    def cur_scale(self):
        return self.loss_scaler.loss_scale

    def get_global_grad_norm(self):
        return None if self._last_norm is None else float(self._last_norm.reshape(-1)[0])

    def _handle_overflow_host(self):
        """fp16 with dynamic loss scaling needs the overflow on the host (one sync per step)."""
        if getattr(self.loss_scaler, "dynamic", False):
            self.overflow = bool(self._skip_t.reshape(-1)[0].item() != 0.0)
            self.loss_scaler.update_scale(self.overflow)
            if self.overflow:
                log_dist(f"overflow: skipping step, loss scale -> {self.loss_scaler.cur_scale}", ranks=[0])
        else:
            self.overflow = False
        return self.overflow
