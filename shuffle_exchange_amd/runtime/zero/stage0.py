"""Plain data parallelism (ZeRO stage 0) with bucketed, overlapped gradient all-reduce.

Parity: reference runtime/engine.py:2170-2184 ``allreduce_gradients`` / :2616-2751
``allreduce_bucket`` / ``buffered_allreduce_fallback`` and runtime/bf16_optimizer.py:35.
Parameters are grouped into flat units of ``bucket_size`` elements (replicated, S = 1); the fp32
gradient accumulator of a unit is all-reduced (``ReduceOp.AVG`` on RCCL) on a side HIP stream as
soon as its last gradient arrives on the accumulation-boundary micro-step, then the fused optimizer
updates fp32 masters and writes the bit16 weights in one pass.

Sparse gradients (``sparse_gradients``: nn.Embedding(sparse=True) weights, marked by the engine;
reference engine.py:2752-2823 ``sparse_allreduce``): each such weight is its own unit; its
gradient stays a sparse (row index, row) tensor through the accumulation micro-steps, and at the
boundary every rank all-gathers the touched rows (sizes first, then padded indices / rows) and
scatter-adds them into the dense fp32 accumulator -- the dense all-reduce result at a fraction of
the bytes when a step touches few rows of a large table.
"""
import torch

from ... import comm as dist
from ...accelerator import get_accelerator
from ...utils.logging import log_dist
from .base import ZeroOptimizerBase
from .flat import FlatUnit, split_into_units
from ..torch_autocast import split_by_comm_dtype, unit_comm_dtype


class DataParallelOptimizer(ZeroOptimizerBase):
    def __init__(self, init_optimizer, *, loss_scaler, clip_grad=0.0, dp_ranks=None, dp_group=None,
                 bucket_size=500_000_000, mp_group=None, shuffle_exchange_cfg=None, fp32_accum=False):
        acc = get_accelerator()
        device = torch.device(acc.current_device_name())
        super().__init__(init_optimizer, loss_scaler, clip_grad, None, overflow_group=None, mp_group=mp_group,
                         device=device)
        self.dp_group = dp_group
        # bf16 without ZeRO accumulates micro-step gradients in fp32 (reference default grad_accum_dtype,
        # engine.py:1081-1085 -> BF16_Optimizer): every micro-step's .grad is added to the unit's fp32
        # accumulator right away instead of accumulating in the bit16 .grad until the boundary
        self.fp32_accum = bool(fp32_accum)
        self.dp_size = len(dp_ranks) if dp_ranks is not None else dist.get_world_size()
        self.comm_stream = acc.named_stream("dp_reduce") if acc.gpu else None
        self.boundary = True
        self.param_unit = {}
        self._hooks = []
        for g, pg in enumerate(init_optimizer.param_groups):
            params = [p for p in pg["params"] if p.requires_grad]
            units = []
            rgroup, rsize = self.dp_group, self.dp_size
            if pg.get("moe", False):  # expert grads: expert-data-parallel group only
                from ...parallel import groups
                name = pg["name"]
                groups.create_expert_and_data_parallel(int(name.rsplit("_", 1)[-1]), name)
                rgroup = groups.get_expert_data_parallel_group(name)
                rsize = groups.get_expert_data_parallel_world_size(name)
            sparse = [p for p in params if getattr(p, "_sxe_sparse", False)]
            dense = [p for p in params if not getattr(p, "_sxe_sparse", False)]
            plists = [pl for run in split_by_comm_dtype(dense) for pl in split_into_units(run, max(1, int(bucket_size)))]
            plists += [[p] for p in sparse]
            for i, plist in enumerate(plists):
                u = FlatUnit(plist, 1, 0, plist[0].dtype, device, name=f"g{g}u{i}", index=i)
                # expert grads are summed over their EDP group and divided by the DENSE dp size
                # (reference engine.py:2713-2716 _reduce_expert_gradients, stage_1_and_2.py:1316)
                u.rgroup, u.rsize, u.rdiv = rgroup, rsize, self.dp_size
                u.comm_dtype = unit_comm_dtype(plist)  # torch_autocast: all-reduce in bf16 / fp16
                u.sparse = getattr(plist[0], "_sxe_sparse", False)
                u.sparse_parts = []
                u.dense_seen = False
                units.append(u)
                for p in plist:
                    self.param_unit[p] = u
            self.units.append(units)
        self._init_master()
        # MoE: expert gradients differ across the expert-parallel group (each rank holds other
        # experts) while dense gradients are identical there after the all-reduce. The norm domain
        # therefore spans the EP group, with dense groups weighted 1/ep so they count once --
        # otherwise ranks clip by different norms and the replicated dense weights drift apart.
        moe_names = sorted({pg["name"] for pg in init_optimizer.param_groups if pg.get("moe", False)})
        if moe_names:
            from ...parallel import groups
            eps = {groups.get_expert_parallel_world_size(n) for n in moe_names}
            if len(eps) > 1:
                raise NotImplementedError("ZeRO-0 with several expert-parallel sizes")
            ep = eps.pop()
            if ep > 1:
                self.extra_norm_group = groups.get_expert_parallel_group(moe_names[0])
                # dense duplicates inside the EP group: its members that are data-parallel peers of
                # this rank (all ep of them, or fewer when the EP group spans the TP ranks)
                ep_ranks = set(groups.get_expert_parallel_ranks(moe_names[0]))
                mine = set(dist.group_ranks(self.dp_group)) if self.dp_group is not None else {dist.get_rank()}
                dup = max(1, len(ep_ranks & mine))
                for pg in init_optimizer.param_groups:
                    if not pg.get("moe", False):
                        pg["norm_weight"] = pg.get("norm_weight", 1.0) / dup
        if hasattr(self.optimizer, "set_segments"):  # layer-wise optimizers (LAMB) on flat masters
            for g, units in enumerate(self.units):
                segs, base = [], 0
                for u in units:
                    segs += [(base + o, n) for o, n in zip(u.offsets, u.numels)]
                    base += u.chunk
                self.optimizer.set_segments(self.master[g], segs)
        for p, u in self.param_unit.items():
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(u)))
        log_dist(f"DP (ZeRO-0): {sum(len(u) for u in self.units)} buckets over {self.dp_size} ranks", ranks=[0])

    def _take_grad(self, u, i, p):
        if u.sparse and p.grad.is_sparse:
            u.sparse_parts.append(p.grad.coalesce())
        else:
            if u.sparse:
                # a sparse-marked weight that received a dense gradient (e.g. an embedding tied to
                # the LM head: sparse + dense = dense): this window's reduce must be the dense one
                u.dense_seen = True
            o, n = u.offsets[i], u.numels[i]
            g = p.grad.to_dense() if p.grad.is_sparse else p.grad
            u.grad[o:o + n].add_(g.reshape(-1))
        p.grad = None

    def grad_ready(self, p):
        """A gradient delivered outside autograd's AccumulateGrad (the FX graph compiler's in-graph
        reduce nodes, compile/fx_backend.py): ``p.grad`` is set; run the per-parameter hook."""
        u = self.param_unit.get(p)
        if u is not None:
            self._make_hook(u)(p)

    def _make_hook(self, u):
        def hook(p):
            if p.grad is None or getattr(p, "_sxe_grad_partial", False):
                return  # partial tile gradient: keep summing in .grad until the last tile
            if not self.boundary:
                if self.fp32_accum:
                    self._take_grad(u, u.param_index[id(p)], p)
                return
            i = u.param_index[id(p)]
            self._take_grad(u, i, p)
            if not u.filled[i]:
                u.filled[i] = True
                u.pending -= 1
                if u.pending == 0:
                    self._allreduce_unit(u)
        return hook

    def _sparse_allreduce_unit(self, u):
        """All-gather the touched rows of a sparse-gradient unit and scatter-add them densely."""
        p = u.params[0]
        rows, width = p.shape[0], p.numel() // p.shape[0]
        dense = u.grad[:u.numel].view(rows, width)
        if u.sparse_parts:
            g = torch.sparse_coo_tensor(torch.cat([t.indices() for t in u.sparse_parts], 1),
                                        torch.cat([t.values() for t in u.sparse_parts], 0), p.shape).coalesce()
            idx, val = g.indices()[0], g.values().reshape(-1, width).to(dense.dtype)
        else:
            idx = torch.zeros(0, dtype=torch.long, device=dense.device)
            val = torch.zeros(0, width, dtype=dense.dtype, device=dense.device)
        u.sparse_parts = []
        if u.rsize == 1:
            dense.index_add_(0, idx, val)
            if self.sp_scale != u.rdiv:
                dense.mul_(self.sp_scale / u.rdiv)
            return
        n = torch.tensor([idx.numel()], dtype=torch.long, device=dense.device)
        ns = [torch.zeros_like(n) for _ in range(u.rsize)]
        dist.all_gather(ns, n, group=u.rgroup)
        ns = [int(x) for x in ns]
        m = max(ns)
        pi = torch.zeros(m, dtype=torch.long, device=dense.device)
        pv = torch.zeros(m, width, dtype=dense.dtype, device=dense.device)
        pi[:idx.numel()].copy_(idx)
        pv[:idx.numel()].copy_(val)
        ai = torch.empty(u.rsize * m, dtype=torch.long, device=dense.device)
        av = torch.empty(u.rsize * m, width, dtype=dense.dtype, device=dense.device)
        dist.all_gather_into_tensor(ai, pi, group=u.rgroup)
        dist.all_gather_into_tensor(av.view(-1), pv.view(-1), group=u.rgroup)
        keep = torch.cat([torch.arange(r * m, r * m + ns[r], device=dense.device) for r in range(u.rsize)])
        dense.index_add_(0, ai[keep], av[keep])
        dense.mul_(self.sp_scale / u.rdiv)

    def _allreduce_unit(self, u):
        if u.sparse and u.dense_seen and u.sparse_parts:
            # mixed window: fold the sparse rows into the dense accumulator, reduce densely
            p = u.params[0]
            g = torch.sparse_coo_tensor(torch.cat([t.indices() for t in u.sparse_parts], 1),
                                        torch.cat([t.values() for t in u.sparse_parts], 0), p.shape).coalesce()
            width = p.numel() // p.shape[0]
            u.grad[:u.numel].view(p.shape[0], width).index_add_(0, g.indices()[0],
                                                                 g.values().reshape(-1, width).to(u.grad.dtype))
            u.sparse_parts = []
        if u.sparse and not u.dense_seen and not u.reduced:
            u.reduced = True
            self._sparse_allreduce_unit(u)
            return
        # 1-bit optimizers past their warm-up synchronise compressed momentum themselves
        if u.reduced or getattr(self.optimizer, "comm_active", False):
            u.reduced = True
            return
        if u.rsize == 1:
            u.reduced = True
            if self.sp_scale != u.rdiv:  # an expert group of one rank still averages over dp
                u.grad.mul_(self.sp_scale / u.rdiv)
            return
        u.reduced = True
        st = self.comm_stream
        if st is not None:
            st.wait_stream(torch.cuda.current_stream())
        with get_accelerator().stream(st):
            g = u.grad if u.comm_dtype is None else u.grad.to(u.comm_dtype)
            if dist.get_backend() == "nccl" and self.sp_scale == 1.0 and u.rdiv == u.rsize:
                dist.all_reduce(g, op=dist.ReduceOp.AVG, group=u.rgroup)
            else:
                dist.all_reduce(g, group=u.rgroup)
                g.mul_(self.sp_scale / u.rdiv)
            if g is not u.grad:
                u.grad.copy_(g)
                if st is not None:
                    g.record_stream(st)

    def set_gradient_accumulation_boundary(self, flag):
        self.boundary = bool(flag)

    def backward_prologue(self):
        for units in self.units:
            for u in units:
                u.begin_backward()
                u.reduced = False

    def reduce_gradients(self, pipeline_parallel=False):
        if not self.boundary:
            return
        for units in self.units:
            for u in units:
                for i, p in enumerate(u.params):
                    if p.grad is not None:
                        self._take_grad(u, i, p)
                self._allreduce_unit(u)

    def step(self, closure=None):
        if self.comm_stream is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)
        coef, skip = self._grad_norm_and_flags()
        if getattr(self.loss_scaler, "dynamic", False) and self._handle_overflow_host():
            self.zero_grad_buffers()
            return
        self._fused_update(coef, skip)
        self.zero_grad_buffers()
        self.global_step += 1

    def zero_grad_buffers(self):
        super().zero_grad_buffers()
        for units in self.units:
            for u in units:
                u.dense_seen = False

    def zero_grad(self, set_to_none=True):
        for p in self.param_unit:
            p.grad = None

    def unit_layout(self, name_of):
        return [[{"params": [name_of.get(p, "") for p in u.params], "shapes": u.shapes, "offsets": u.offsets,
                  "numel": u.numel, "padded": u.padded, "chunk": u.chunk} for u in units] for units in self.units]

    def state_dict(self):
        return {"loss_scaler": self.loss_scaler.state_dict(), "clip_grad": self.clip_grad,
                "base_optimizer_state": self.optimizer.state_dict(),
                "single_partition_of_fp32_groups": [m.data for m in self.master], "zero_stage": 0,
                "ds_version": "sxe-0.1"}

    def load_state_dict(self, sd, load_optimizer_states=True, load_from_fp32_weights=True):
        self.loss_scaler.load_state_dict(sd["loss_scaler"])
        if load_optimizer_states:
            self.optimizer.load_state_dict(sd["base_optimizer_state"])
        for m, s in zip(self.master, sd["single_partition_of_fp32_groups"]):
            m.data.copy_(s.to(m.device))
        for units in self.units:
            for u in units:
                u.shard.copy_(u.master)
