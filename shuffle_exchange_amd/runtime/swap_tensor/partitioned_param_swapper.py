"""ZeRO-Infinity parameter tier on NVMe: every non-persistent ZeRO-3 unit's bit16 shard lives in a
swap file and is read into one of a small pool of pinned host buffers only around its gather.

Parity: reference runtime/swap_tensor/partitioned_param_swapper.py:37
``AsyncPartitionedParameterSwapper`` (``swap_in`` :291, ``swap_out_and_release`` :274,
``synchronize_reads`` :243, buffer pool :90-112, ``buffer_count`` / ``buffer_size`` of the
``offload_param`` config). MI355X-first differences:

* The swap granule is the ZeRO-3 *unit* (one flat bit16 shard per module unit, runtime/zero/flat.py),
  so one read is one contiguous 4 KiB-aligned extent per unit -- the whole-extent O_DIRECT path of
  the AIO engine (csrc/include/sxe_aio_core.h), split into ``block_size`` pieces over its threads.
* Reads are issued ahead along the recorded fetch order (``prefetch``), into pinned buffers that the
  HIP all-gather stream then copies to HBM asynchronously; a buffer returns to the pool when the
  event recorded after that copy has completed (``release``), never by a device-wide sync.
* The optimizer step writes the updated bit16 shard straight into a pool buffer (``stage``) that is
  written back asynchronously (``commit``): parameters never need a host-RAM mirror, so the
  trainable model size is bounded by NVMe capacity, not by host RAM.
"""
import os

import torch

from ...utils.logging import log_dist

ALIGN = 4096


class AsyncPartitionedParameterSwapper:
    """A write-back cache of unit shards over one swap file, with a pool of pinned buffers.

    Per unit key: not resident / resident in buffer i (read possibly pending, ``dirty`` when it may
    differ from the file, ``pins`` while a HIP copy reads it). ``acquire``/``release`` bracket a
    gather; ``access`` hands out the resident buffer for arbitrary (possibly in-place) use and marks
    it dirty; ``overwrite`` does the same without reading the old contents first; ``flush`` writes
    every dirty buffer back. Eviction takes the least recently used unpinned buffer, writing it back
    first if dirty and waiting for the HIP event of its last reader."""

    _count = 0

    def __init__(self, nvme_path, rank, dtype, aio_config=None, buffer_count=5):
        from ...ops.aio import AsyncIOHandle
        assert nvme_path, "offload_param.device=nvme needs nvme_path"
        self.dir = os.path.join(nvme_path, f"sxe_param_swap_rank{rank}")
        os.makedirs(self.dir, exist_ok=True)
        # one file per swapper instance (several engines may share an nvme_path in one process)
        AsyncPartitionedParameterSwapper._count += 1
        self.file = os.path.join(self.dir, f"params_{os.getpid()}_{AsyncPartitionedParameterSwapper._count}.swp")
        open(self.file, "wb").close()
        self.dtype = dtype
        self.esize = torch.tensor([], dtype=dtype).element_size()
        a = aio_config
        kw = dict(block_size=getattr(a, "block_size", 1 << 20), queue_depth=getattr(a, "queue_depth", 8),
                  intra_op_parallelism=max(2, getattr(a, "intra_op_parallelism", 1) or 1))
        self.rd = AsyncIOHandle(**kw)
        self.wr = AsyncIOHandle(**kw)
        self.offset, self.numel = {}, {}
        self._end = 0
        self.buffer_count = max(2, int(buffer_count))
        self.buffers = []      # allocated at first use: sized by the largest registered shard
        self.free = []
        self.where = {}        # key -> buffer index (resident)
        self.key_of = {}       # buffer index -> key
        self.reads = {}        # key -> pending AIO read request
        self.writes = {}       # buffer index -> pending AIO write request
        self.fence = {}        # buffer index -> HIP event of its last reader
        self.dirty = set()     # keys whose buffer may differ from the file
        self.pins = {}         # key -> active readers
        self.lru = []          # resident keys, least recently used first
        self.bytes_read = 0
        self.bytes_written = 0

    # ------------------------------------------------------------------------------ layout
    def _slot_elems(self, n):
        return (n * self.esize + ALIGN - 1) // ALIGN * ALIGN // self.esize

    def _extent(self, key):
        return self.offset[key], self._slot_elems(self.numel[key])

    def register(self, key, src):
        """Reserve `key`'s extent and write its initial contents (a host or device tensor)."""
        n = src.numel()
        self.offset[key] = self._end
        self.numel[key] = int(n)
        self._end += self._slot_elems(n) * self.esize
        tmp = torch.zeros(self._slot_elems(n), dtype=self.dtype)
        tmp[:n].copy_(src.reshape(-1))
        self.wr.wait_request(self.wr.async_pwrite(tmp, self.file, self.offset[key]))
        self.bytes_written += tmp.numel() * self.esize

    def _alloc(self):
        from ..zero.offload import pinned_empty
        elems = self._slot_elems(max(self.numel.values()))
        self.buffers = [pinned_empty(elems, self.dtype) for _ in range(self.buffer_count)]
        self.free = list(range(self.buffer_count))
        log_dist(f"ZeRO-Infinity: {len(self.numel)} parameter shards on NVMe under {self.dir}; "
                 f"{self.buffer_count} pinned swap buffers of {elems * self.esize / 2**20:.1f} MiB", ranks=[0])

    # ------------------------------------------------------------------------------ buffers
    def _touch(self, key):
        if key in self.lru:
            self.lru.remove(key)
        self.lru.append(key)

    def _quiesce(self, i):
        ev = self.fence.pop(i, None)
        if ev is not None:
            ev.synchronize()
        req = self.writes.pop(i, None)
        if req is not None:
            self.wr.wait_request(req)

    def _write_back(self, key):
        i = self.where[key]
        off, n = self._extent(key)
        if n > self.numel[key]:
            self.buffers[i][self.numel[key]:n].zero_()
        self.writes[i] = self.wr.async_pwrite(self.buffers[i][:n], self.file, off)
        self.bytes_written += n * self.esize
        self.dirty.discard(key)

    def _evict(self, key):
        i = self.where[key]
        req = self.reads.pop(key, None)
        if req is not None:
            self.rd.wait_request(req)
        if key in self.dirty:
            self._write_back(key)
        self._quiesce(i)
        del self.where[key], self.key_of[i]
        self.lru.remove(key)
        return i

    def _take_buffer(self, block=True):
        if not self.buffers:
            self._alloc()
        if self.free:
            i = self.free.pop()
            self._quiesce(i)
            return i
        for key in self.lru:  # least recently used first
            if self.pins.get(key, 0) == 0:
                i = self.where[key]
                if not block and (key in self.dirty or key in self.reads
                                  or (i in self.fence and not self.fence[i].query())):
                    continue  # read-ahead never waits on another unit's copy or write-back
                return self._evict(key)
        if block:
            raise RuntimeError("NVMe parameter swapper: every buffer is pinned by an in-flight gather; "
                               "raise offload_param.buffer_count")
        return None

    def _resident(self, key, read=True, block=True):
        if key in self.where:
            self._touch(key)
            return True
        i = self._take_buffer(block)
        if i is None:
            return False
        self.where[key], self.key_of[i] = i, key
        self._touch(key)
        if read:
            off, n = self._extent(key)
            self.reads[key] = self.rd.async_pread(self.buffers[i][:n], self.file, off)
            self.bytes_read += n * self.esize
        return True

    def _view(self, key):
        req = self.reads.pop(key, None)
        if req is not None:
            self.rd.wait_request(req)
        return self.buffers[self.where[key]][:self.numel[key]]

    # ------------------------------------------------------------------------------ API
    def prefetch(self, key):
        """Start reading `key`'s shard if a buffer is available without waiting."""
        self._resident(key, read=True, block=False)

    def acquire(self, key):
        """The shard as a pinned host tensor for a reader; pinned until ``release``."""
        self._resident(key)
        self.pins[key] = self.pins.get(key, 0) + 1
        return self._view(key)

    def release(self, key, event=None):
        """The reader is enqueued; `event` (recorded after its HIP copy) guards buffer reuse."""
        self.pins[key] -= 1
        if event is not None:
            self.fence[self.where[key]] = event

    def access(self, key):
        """The resident shard for arbitrary use (in-place writes allowed): marked dirty."""
        self._resident(key)
        self.dirty.add(key)
        return self._view(key)

    def overwrite(self, key):
        """A buffer to write the whole new shard into (old contents not read): marked dirty."""
        if key not in self.where:
            self._resident(key, read=False)
        self.dirty.add(key)
        return self._view(key)

    def read_copy(self, key):
        """A standalone host copy of the shard (checkpointing); does not mark it dirty."""
        self._resident(key)
        return self._view(key).clone()

    def flush(self):
        """Write every dirty shard back and wait for all I/O."""
        for key in list(self.dirty):
            self._write_back(key)
        self.rd.wait()
        self.wr.wait()
        self.reads.clear()
        self.writes.clear()

    def synchronize_reads(self):
        self.rd.wait()
        self.reads.clear()

    def close(self):
        """Drain all I/O and delete the swap file."""
        try:
            self.rd.wait()
            self.wr.wait()
            os.remove(self.file)
        except (OSError, RuntimeError):
            pass

    def __del__(self):
        self.close()
