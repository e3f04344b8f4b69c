"""Flat parameter units: the memory layout shared by ZeRO-1/2/3 on MI355X.

A *unit* is a set of parameters laid out back-to-back in ONE bit16 buffer, padded so it splits
into ``S`` equal, 256-byte-aligned chunks (S = ZeRO group size). Rank ``r`` of the group owns chunk
``r`` of every unit. Consequences (the MI355X-first design choice vs. the reference):

* gradient reduction of a unit is ONE true ``reduce_scatter_tensor`` of the contiguous unit
  buffer straight into the owner's chunk -- the reference's ZeRO-2 default instead all-reduces each
  bucket and lets the owner copy its slice (stage_1_and_2.py:1189-1204 with
  use_multi_rank_bucket_allreduce=True), 2x the xGMI traffic;
* the post-step parameter rebuild is ONE ``all_gather_into_tensor`` per unit (in place);
* units are sized to the bucket size (ZeRO-1/2) or to a module (ZeRO-3), so every collective is a
  large contiguous message (>= tens of MB amortise RCCL launch latency over 7 xGMI links).

The fp32 master chunks of all units of a parameter group are contiguous in one buffer so the
optimizer runs as one multi-tensor launch that also writes the bit16 chunk back.
"""
import math

import torch

ALIGN_BYTES = 256


def _align_elems(dtype):
    return ALIGN_BYTES // torch.tensor([], dtype=dtype).element_size()


class FlatUnit:
    def __init__(self, params, group_size, rank_in_group, dtype, device, name="", index=0,
                 materialize_full=True):
        self.params = list(params)
        self.name = name
        self.index = index
        self.S = group_size
        self.rank = rank_in_group
        self.dtype = dtype
        self.device = device
        # zero.Init-partitioned parameters carry their logical shape in ds_shape (p.data is empty)
        self.shapes = [tuple(getattr(p, "ds_shape", p.shape)) for p in self.params]
        self.numels = [math.prod(s) for s in self.shapes]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.numel = off
        a = _align_elems(dtype) * self.S
        self.padded = max(a, int(math.ceil(self.numel / a)) * a)
        self.chunk = self.padded // self.S
        self.lo = self.rank * self.chunk
        self.hi = self.lo + self.chunk
        self.flat = None           # full bit16 buffer (stage 1/2 always; stage 3 while fetched)
        self.swap = None           # NVMe parameter tier (ZeRO-Infinity): the shard lives in a swap file
        self.shard = None          # this rank's chunk (a view of `flat` for stage 1/2; own storage stage 3)
        self.master = None         # fp32 chunk (view into the group master buffer)
        self.grad = None           # fp32 chunk gradient accumulator (view into group grad buffer)
        self.staging = None        # full-size grad staging buffer during backward
        self.staging_dtype = None  # None: the unit dtype; fp32 when gradients carry across micro-steps
        self.comm_dtype = None     # gradient-reduction dtype override (torch_autocast units)
        self.carry = False         # staging already holds earlier micro-steps' gradients (deferred RS)
        self.filled = None         # per-param "grad copied to staging" flags
        self.pending = 0
        self.param_index = {id(p): i for i, p in enumerate(self.params)}
        if materialize_full:
            self._build_full()

    # ------------------------------------------------------------------------------------------
    @property
    def shard(self):
        """This rank's bit16 chunk. With the NVMe tier: the swap cache's resident pinned buffer,
        read in on demand and marked dirty (any in-place edit is written back on eviction/flush)."""
        if self.swap is not None:
            return self.swap.access(self)
        return self._shard

    @shard.setter
    def shard(self, v):
        self._shard = v

    def shard_for_overwrite(self):
        """The chunk to receive a whole new value (optimizer step): no swap-in read first."""
        if self.swap is not None:
            return self.swap.overwrite(self)
        return self._shard

    def shard_is_cuda(self):
        return self.swap is None and self._shard is not None and self._shard.is_cuda

    def _build_full(self):
        flat = torch.zeros(self.padded, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                flat[o:o + n].copy_(p.data.reshape(-1))
        self.flat = flat
        self.link_params()
        self.shard = flat[self.lo:self.hi]

    def link_params(self):
        """Point every parameter's storage at its slot in ``flat``."""
        for p, o, n, s in zip(self.params, self.offsets, self.numels, self.shapes):
            p.data = self.flat[o:o + n].view(s)
            p.ds_shape, p.ds_numel = torch.Size(s), n

    def unlink_params(self):
        """Released (ZeRO-3) unit: every parameter becomes an empty tensor -- as in the reference,
        reading a released parameter yields numel 0 (``ds_shape`` keeps the logical shape)
        instead of a view into freed memory, which on the GPU would be an illegal access."""
        empty = self.flat.new_empty(0)
        for p in self.params:
            p.data = empty

    def param_range_in_shard(self, i):
        """Intersection of param i with this rank's chunk: (param_lo, param_hi, shard_lo) or None."""
        o, n = self.offsets[i], self.numels[i]
        lo, hi = max(o, self.lo), min(o + n, self.hi)
        if lo >= hi:
            return None
        return lo - o, hi - o, lo - self.lo

    def begin_backward(self):
        self.pending = len(self.params)
        self.filled = [False] * len(self.params)

    def stage_grad(self, p, grad):
        if grad.is_sparse:  # nn.Embedding(sparse=True) under ZeRO: reduced densely with its unit
            grad = grad.to_dense()
        i = self.param_index[id(p)]
        if self.staging is None:
            self.staging = torch.empty(self.padded, dtype=self.staging_dtype or self.dtype, device=self.device)
            if self.padded > self.numel:
                self.staging[self.numel:].zero_()
        o, n = self.offsets[i], self.numels[i]
        if self.filled[i] or self.carry:
            self.staging[o:o + n].add_(grad.reshape(-1))
            if not self.filled[i]:
                self.filled[i] = True
                self.pending -= 1
        else:
            self.staging[o:o + n].copy_(grad.reshape(-1))
            self.filled[i] = True
            self.pending -= 1
        return self.pending == 0

    def fill_missing(self):
        """Zero the staging slots of parameters that received no gradient this backward."""
        if self.staging is None:
            self.staging = torch.zeros(self.padded, dtype=self.staging_dtype or self.dtype, device=self.device)
        elif not self.carry:  # carried slots hold earlier micro-steps' sums: nothing to zero
            for i, f in enumerate(self.filled):
                if not f:
                    o, n = self.offsets[i], self.numels[i]
                    self.staging[o:o + n].zero_()
        self.pending = 0
        self.filled = [True] * len(self.params)


def split_into_units(params, max_elems):
    """Greedy split of an ordered param list into units of at most `max_elems` elements (a single
    larger parameter forms its own unit)."""
    units, cur, cur_n = [], [], 0
    for p in params:
        n = p.numel()
        if cur and cur_n + n > max_elems:
            units.append(cur)
            cur, cur_n = [], 0
        cur.append(p)
        cur_n += n
    if cur:
        units.append(cur)
    return units
