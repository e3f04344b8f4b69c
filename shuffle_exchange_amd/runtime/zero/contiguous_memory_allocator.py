"""Defragmenting allocator over one pre-allocated buffer (reference
runtime/zero/contiguous_memory_allocator.py:16 ``ContiguousMemoryAllocator``).

ZeRO here lays parameters out in flat units up front, so the stage-3 hot path never needs this; it
is provided for code that manages its own pool (e.g. swapping buffers): ``allocate_tensor(n)``
returns a view into the pool, ``release_tensor(t)`` frees it, and when no single free range is large
enough but the total is, live tensors are compacted towards the start of the pool (their ``.data``
and that of parameters assigned into them is re-pointed, as in the reference) before allocating.
"""
import torch


class ContiguousMemoryAllocator:
    def __init__(self, size, dtype, device):
        self.buffer = torch.zeros(size, dtype=dtype, device=device)
        self.size = size
        self.total_free = size
        self.largest_contiguous = size
        self.max_allocated = 0
        self.contiguous_sizes = {0: size}  # free ranges: start -> length
        self.tensor_addresses = {}  # id -> start
        self.tensor_sizes = {}  # id -> numel
        self.tensor_map = {}  # id -> tensor view
        self.id_to_params = {}  # id -> [(param, numel, shape)]
        self._next_id = 0

    # -------------------------------------------------------------------------------- public API
    def allocate_tensor(self, size):
        assert size <= self.total_free, f"not enough memory: need {size}, free {self.total_free}"
        if self.largest_contiguous < size:
            self._defragment_memory()
        start = self._first_fit(size)
        self._mark_used(start, size)
        tid = self._next_id
        self._next_id += 1
        t = self.buffer.narrow(0, start, size)
        t._sxe_alloc_id = tid
        self.tensor_addresses[tid], self.tensor_sizes[tid], self.tensor_map[tid] = start, size, t
        self.total_free -= size
        self.max_allocated = max(self.max_allocated, self.size - self.total_free)
        self._update_largest()
        return t

    def assign_to_param(self, tensor, param, numel, shape):
        tid = tensor._sxe_alloc_id
        assert numel <= self.tensor_sizes[tid]
        param.data = tensor.narrow(0, 0, numel).view(shape)
        self.id_to_params.setdefault(tid, []).append((param, numel, shape))

    def release_tensor(self, tensor):
        self._release(tensor._sxe_alloc_id)

    def release_tensor_with_id(self, tid):
        self._release(tid)

    def print_allocation(self, resolution=200):
        chars = ["."] * resolution
        for tid, start in self.tensor_addresses.items():
            a = start * resolution // self.size
            b = max(a + 1, (start + self.tensor_sizes[tid]) * resolution // self.size)
            for i in range(a, min(b, resolution)):
                chars[i] = "|"
        print("".join(chars))

    def max_allocated_memory(self):
        return self.max_allocated

    # ------------------------------------------------------------------------------- internals
    def _first_fit(self, size):
        for start in sorted(self.contiguous_sizes):
            if self.contiguous_sizes[start] >= size:
                return start
        raise RuntimeError("allocator invariant broken: no free range after defragmentation")

    def _mark_used(self, start, size):
        length = self.contiguous_sizes.pop(start)
        if length > size:
            self.contiguous_sizes[start + size] = length - size

    def _release(self, tid):
        start, size = self.tensor_addresses.pop(tid), self.tensor_sizes.pop(tid)
        self.tensor_map.pop(tid)
        self.id_to_params.pop(tid, None)
        self.total_free += size
        self.contiguous_sizes[start] = size
        self._coalesce()
        self._update_largest()

    def _coalesce(self):
        merged, cur = {}, None
        for s in sorted(self.contiguous_sizes):
            n = self.contiguous_sizes[s]
            if cur is not None and cur + merged[cur] == s:
                merged[cur] += n
            else:
                merged[s] = n
                cur = s
        self.contiguous_sizes = merged

    def _update_largest(self):
        self.largest_contiguous = max(self.contiguous_sizes.values(), default=0)

    def _defragment_memory(self):
        """Slide every live tensor down to the lowest free address, in address order (each
        destination lies below its source, so no not-yet-moved tensor is overwritten)."""
        dst = 0
        for tid in sorted(self.tensor_addresses, key=self.tensor_addresses.get):
            src, n = self.tensor_addresses[tid], self.tensor_sizes[tid]
            if src != dst:
                self.buffer.narrow(0, dst, n).copy_(self.buffer.narrow(0, src, n).clone())
                view = self.buffer.narrow(0, dst, n)
                self.tensor_map[tid].data = view
                self.tensor_addresses[tid] = dst
                for param, numel, shape in self.id_to_params.get(tid, []):
                    param.data = view.narrow(0, 0, numel).view(shape)
            dst += n
        self.contiguous_sizes = {dst: self.size - dst} if dst < self.size else {}
        self._update_largest()
