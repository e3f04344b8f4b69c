"""Shuffle-exchange: hierarchical ZeRO with inter-slice parameter averaging (the fork's feature).

Semantics (reference runtime/zero/stage_1_and_2.py:163-241, 692-734, 2092-2250):
the ZeRO data-parallel group of W ranks is cut into W/S *slices* of S consecutive ranks. ZeRO
partitioning, gradient reduce-scatter, grad-norm and the parameter all-gather all happen INSIDE a
slice. After each optimizer step the bit16 chunk a rank owns is synchronised with the ranks that
own the same chunk offset in the other slices, by one of four methods:

``RR``      exact mean over all slices (one all-reduce per offset group).
``shuffle`` mean inside random groups ("rings") of W/(S*rings) slices; the grouping is redrawn every
            ``shuffle_step`` calls of ``shuffle_exchange()``.
``H-RR``    two-level mean: reduce to the ring leader, all-reduce between the 2 leaders, broadcast.
``Gossip``  push-sum style: random senders halve their weight ``alpha`` and push (alpha, chunk) to a
            random peer, which merges weighted messages before its next step.

Only the bit16 working copy is averaged; fp32 masters and optimizer moments stay slice-local (the
reference's behaviour; ``average_master=True`` additionally averages the fp32 chunk -- new).

MI355X-first differences, each a fix or a cost the reference pays per step:
* communicators are created ONCE per distinct rank set and cached (the reference destroys and
  re-creates every RCCL communicator on each reshuffle, stage_1_and_2.py:698-711);
* all rank-shared randomness (shuffle permutation, Gossip senders/destinations) comes from a
  dedicated ``torch.Generator`` seeded identically on every rank, so it cannot diverge with
  model-side RNG use (the reference relies on the global torch RNG being in lock-step);
* means are exact-divided: with a power-of-two member count the pre-division of a bit16 chunk is an
  exponent shift (no rounding) and only the summation rounds -- pinned against the fp32 mean in
  tests/test_shuffle_exchange_w8.py; other counts average in fp32 (upcast, sum, divide, round once);
* Gossip sends exactly-sized buffers with ``batch_isend_irecv`` (the reference receives into an
  8 GB 4e9-element buffer regardless of the tensor size, stage_1_and_2.py:2190-2194) and keeps
  ``alpha`` in fp32 so the push-sum mass is conserved to fp32 precision;
* invalid shapes (W % S != 0, slices % rings != 0) raise instead of logging and continuing with a
  zero world size (stage_1_and_2.py:179-180).
"""
import torch
import torch.distributed as tdist

from ... import comm as dist
from ...utils.logging import log_dist


class SliceTopology:
    """Slices of `slice_count` consecutive ranks inside the ZeRO data-parallel rank list."""

    def __init__(self, dp_ranks, slice_count):
        self.dp_ranks = list(dp_ranks)
        W = len(self.dp_ranks)
        S = int(slice_count)
        if S < 1 or W % S != 0:
            raise ValueError(f"shuffle_exchange: slice_count={S} must divide the data-parallel world size {W}")
        self.W, self.S = W, S
        self.num_slices = W // S
        me = dist.get_rank()
        self.dp_index = self.dp_ranks.index(me)
        self.slice_id = self.dp_index // S
        self.offset = self.dp_index % S
        self.slice_group = None
        self.slice_ranks = None
        for g in range(self.num_slices):
            ranks = self.dp_ranks[g * S:(g + 1) * S]
            pg = dist.new_group(ranks)
            if me in ranks:
                self.slice_group, self.slice_ranks = pg, ranks

    def make_reduce_groups(self):
        """A second communicator per slice (collective: every rank creates every slice's), for
        gradient reduction that must run concurrently with the parameter all-gathers on
        ``slice_group``."""
        if getattr(self, "reduce_group", None) is not None or self.S == 1:
            return getattr(self, "reduce_group", None)
        me = dist.get_rank()
        self.reduce_group = None
        for g in range(self.num_slices):
            ranks = self.dp_ranks[g * self.S:(g + 1) * self.S]
            pg = dist.new_group(ranks, tag="zero_reduce")
            if me in ranks:
                self.reduce_group = pg
        return self.reduce_group

    def real(self, slice_idx, offset=None):
        return self.dp_ranks[slice_idx * self.S + (self.offset if offset is None else offset)]

    def offset_groups(self, slice_ids):
        """Create (collectively, on every rank) one group per offset over `slice_ids`; return mine
        (or None if my slice is not in `slice_ids`)."""
        mine = None
        slice_ids = list(slice_ids)
        for o in range(self.S):
            ranks = [self.real(s, o) for s in slice_ids]
            pg = dist.new_group(ranks)
            if self.slice_id in slice_ids and o == self.offset:
                mine = (pg, ranks)
        return mine


class ShuffleExchange:
    def __init__(self, topo: SliceTopology, method="RR", rings=8, shuffle_step=50, seed=1234, gossip_p=1.0,
                 average_master=False):
        self.topo = topo
        self.comm_device = None  # set by ZeRO-3 so host-resident shards are reduced on the device
        self.method = method
        self.shuffle_step = max(1, int(shuffle_step))
        self.seed = int(seed)
        self.gossip_p = float(gossip_p)
        self.average_master = average_master
        self.batch_count = 0
        self.reshuffles = 0
        self.group = None
        self.group_ranks = None
        n = topo.num_slices
        self.active = n > 1
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(self.seed)
        if not self.active:
            return
        if method == "RR":
            self.group, self.group_ranks = topo.offset_groups(range(n))
        elif method == "shuffle":
            self.rings = self._check_rings(rings)
            rs = n // self.rings
            for i in range(self.rings):
                g = topo.offset_groups(range(i * rs, (i + 1) * rs))
                if g is not None:
                    self.group, self.group_ranks = g
        elif method == "H-RR":
            if n % 2 != 0:
                raise ValueError(f"H-RR needs an even number of slices, got {n}")
            self.rings = 2
            rs = n // 2
            for start in (0, rs):
                g = topo.offset_groups(range(start, start + rs))
                if g is not None:
                    self.group, self.group_ranks = g
            top = [0, rs]
            self.top_node = topo.real(rs * (topo.slice_id // rs))
            tg = topo.offset_groups(top)
            self.in_top = topo.slice_id in top
            self.top_group, self.top_ranks = tg if tg is not None else (None, None)
        elif method == "Gossip":
            self.alpha = torch.tensor(1.0 / n, dtype=torch.float32)
            self.queue = []
        else:
            raise ValueError(f"unknown shuffle-exchange method {method}")

    # -------------------------------------------------------------------------------------------
    def _check_rings(self, rings):
        n = self.topo.num_slices
        rings = int(rings)
        if rings > n:
            log_dist(f"shuffle_exchange: rings={rings} > slices={n}; using rings={n}", ranks=[0])
            rings = n
        if rings < 1 or n % rings != 0:
            raise ValueError(f"shuffle_exchange: rings={rings} must divide the number of slices {n}")
        return rings

    @staticmethod
    def _mean_allreduce(t, group, n):
        if n & (n - 1) == 0 or t.dtype == torch.float32:
            t.div_(n)  # exact for a power-of-two n
            dist.all_reduce(t, group=group)
        else:
            f = t.float().div_(n)
            dist.all_reduce(f, group=group)
            t.copy_(f)

    def _packed(self, tensors, fn):
        """Run ``fn(flat)`` once per dtype over all ``tensors`` packed back to back: one collective per
        step instead of one per chunk (every RCCL call pays its launch + ring-setup latency over the
        xGMI links; the pack / unpack copies run at HBM speed). A lone tensor goes in place. The pack
        buffer is persistent per (dtype, device): no allocation per step (the chunks themselves cannot
        alias one buffer -- each unit's flat buffer must stay contiguous for its all-gather)."""
        by_dt = {}
        for t in tensors:
            by_dt.setdefault(t.dtype, []).append(t)
        bufs = self.__dict__.setdefault("_pack_bufs", {})
        cdev = self.comm_device
        for ts in by_dt.values():
            dev = ts[0].device if cdev is None else cdev
            on_dev = all(t.device == dev for t in ts)
            if len(ts) == 1 and ts[0].is_contiguous() and on_dev:
                fn(ts[0])
                continue
            total = sum(t.numel() for t in ts)
            key = (ts[0].dtype, dev)
            buf = bufs.get(key)
            if buf is None or buf.numel() < total:
                buf = bufs[key] = torch.empty(total, dtype=ts[0].dtype, device=dev)
            flat = buf[:total]
            if on_dev:
                torch.cat([t.reshape(-1) for t in ts], out=flat)
            else:  # host-resident shards (ZeRO-3 offload_param): H2D into the pack buffer, D2H back
                o = 0
                for t in ts:
                    flat[o:o + t.numel()].copy_(t.reshape(-1), non_blocking=True)
                    o += t.numel()
            fn(flat)
            o = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[o:o + n].view_as(t))
                o += n

    # -------------------------------------------------------------------------------------------
    def shuffle_exchange(self):
        """User hook (reference stage_1_and_2.py:692): reshuffle every `shuffle_step` calls."""
        if self.method != "shuffle" or not self.active:
            return
        self.batch_count += 1
        if self.batch_count % self.shuffle_step == 0:
            self._shuffle()

    def _shuffle(self):
        n = self.topo.num_slices
        self.reshuffles += 1
        perm = torch.randperm(n, generator=self.gen).view(self.rings, -1).tolist()
        self.group, self.group_ranks = None, None
        for slices in perm:
            g = self.topo.offset_groups(slices)  # cached per rank set: no RCCL re-init when seen before
            if g is not None:
                self.group, self.group_ranks = g

    def reset_rings(self, rings):
        if self.method != "shuffle" or not self.active:
            return
        self.rings = self._check_rings(rings)
        self._shuffle()
        self.batch_count = 0

    def current_groups(self):
        return self.group_ranks

    # -------------------------------------------------------------------------------------------
    def pre_step(self, shards):
        """Gossip: merge queued (alpha, chunk) messages into the local chunks before the step
        (reference stage_1_and_2.py:2092-2108)."""
        if self.method != "Gossip" or not self.active or not self.queue:
            return
        for alpha_m, chunks in self.queue:
            a = float(self.alpha)
            am = float(alpha_m)
            for t, c in zip(shards, chunks):
                t.mul_(a / (a + am)).add_(c.to(t.device, t.dtype), alpha=am / (a + am))
            self.alpha += am
        self.queue = []

    def sync(self, shards, masters=None):
        """Post-step inter-slice synchronisation of this rank's bit16 chunks (list of tensors)."""
        if not self.active:
            return
        tensors = list(shards) + (list(masters) if (self.average_master and masters is not None) else [])
        m = self.method
        if m == "RR":
            self._packed(tensors, lambda t: self._mean_allreduce(t, self.group, self.topo.num_slices))
        elif m == "shuffle":
            self._packed(tensors, lambda t: self._mean_allreduce(t, self.group, len(self.group_ranks)))
        elif m == "H-RR":
            # sum up the hierarchy, divide ONCE at the top (pre-dividing every bit16 chunk by n
            # before the sums would round each contribution in bf16 first)
            n = self.topo.num_slices

            def hrr(t):
                dist.reduce(t, dst=self.top_node, group=self.group)
                if self.in_top:
                    dist.all_reduce(t, group=self.top_group)
                    t.div_(n)
                dist.broadcast(t, src=self.top_node, group=self.group)
            self._packed(tensors, hrr)
        elif m == "Gossip":
            self._gossip(shards)

    def _gossip(self, shards):
        n = self.topo.num_slices
        # the step's whole plan in two draws (host generator, one .tolist() each): who sends, and to whom
        senders = torch.bernoulli(torch.full((n,), self.gossip_p), generator=self.gen).tolist()
        dests = torch.randint(0, n, (n,), generator=self.gen).tolist()
        me = self.topo.slice_id
        ops, recv = [], []
        dev = shards[0].device if self.comm_device is None else self.comm_device
        for sid in range(n):
            dest = int(dests[sid])
            if senders[sid] != 1 or dest == sid:
                continue
            if sid == me:
                self.alpha /= 2
                a = self.alpha.reshape(1).to(dev)
                peer = self.topo.real(dest)
                ops.append(dist.P2POp(tdist.isend, a, peer))
                for t in shards:
                    ops.append(dist.P2POp(tdist.isend, t.to(dev).contiguous(), peer))
            if dest == me:
                a = torch.empty(1, dtype=torch.float32, device=dev)
                bufs = [torch.empty(t.shape, dtype=t.dtype, device=dev) for t in shards]
                peer = self.topo.real(sid)
                ops.append(dist.P2POp(tdist.irecv, a, peer))
                for b in bufs:
                    ops.append(dist.P2POp(tdist.irecv, b, peer))
                recv.append((a, bufs))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        for a, bufs in recv:
            self.queue.append((a.cpu().reshape(()), bufs))

    def synchronization(self, shards):
        """World mean of the parameters (reference stage_1_and_2.py:722-728): for shuffle and
        Gossip only. The chunks of one offset across all slices are averaged; the caller then
        all-gathers inside the slice, which equals the reference's full-flat world all-reduce."""
        if self.method not in ("shuffle", "Gossip") or not self.active:
            return False
        if not hasattr(self, "_world_offset_group"):
            self._world_offset_group = self.topo.offset_groups(range(self.topo.num_slices))[0]
        self._packed(list(shards), lambda t: self._mean_allreduce(t, self._world_offset_group, self.topo.num_slices))
        return True

    def state_dict(self):
        return {"method": self.method, "batch_count": self.batch_count, "reshuffles": self.reshuffles,
                "gen": self.gen.get_state(), "alpha": float(getattr(self, "alpha", 0.0)),
                "rings": getattr(self, "rings", None)}

    def load_state_dict(self, sd):
        self.batch_count = sd.get("batch_count", 0)
        self.gen.set_state(sd["gen"])
        if self.method == "Gossip" and "alpha" in sd:
            self.alpha = torch.tensor(sd["alpha"], dtype=torch.float32)
        if self.method == "shuffle" and self.active and sd.get("reshuffles", 0) > 0:
            # replay the same permutation the saving run ended on
            self.gen.manual_seed(self.seed)
            self.reshuffles = 0
            for _ in range(sd["reshuffles"]):
                self._shuffle()
            self.gen.set_state(sd["gen"])
