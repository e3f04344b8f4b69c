"""Async tensor <-> file I/O (parity: reference ops/aio + csrc/aio/py_lib aio_handle API).

``AsyncIOHandle(block_size, queue_depth, single_submit, overlap_events, intra_op_parallelism)``
wraps the C++ thread-pool engine ``torch.classes.sxe_cpu.AioHandle`` (csrc/cpu/aio.cpp).
Buffers must be contiguous host tensors; pinned buffers (``new_cpu_locked_tensor``) let the
same staging memory feed the GPU through DMA without another copy.
"""
import torch

from . import native


class AsyncIOHandle:
    def __init__(self, block_size=1 << 20, queue_depth=32, single_submit=False, overlap_events=True,
                 intra_op_parallelism=4):
        native.require_cpu()
        self._h = torch.classes.sxe_cpu.AioHandle(int(block_size), int(queue_depth), bool(single_submit),
                                                  bool(overlap_events), int(intra_op_parallelism))

    def async_pwrite(self, buffer, filename, file_offset=0):
        return self._h.async_pwrite(buffer, str(filename), int(file_offset))

    def async_pread(self, buffer, filename, file_offset=0):
        return self._h.async_pread(buffer, str(filename), int(file_offset))

    def sync_pwrite(self, buffer, filename, file_offset=0):
        return self._h.sync_pwrite(buffer, str(filename), int(file_offset))

    def sync_pread(self, buffer, filename, file_offset=0):
        return self._h.sync_pread(buffer, str(filename), int(file_offset))

    # reference spellings
    def read(self, buffer, filename, async_op=False):
        return (self.async_pread if async_op else self.sync_pread)(buffer, filename)

    def write(self, buffer, filename, async_op=False):
        return (self.async_pwrite if async_op else self.sync_pwrite)(buffer, filename)

    def wait(self):
        return self._h.wait()

    def wait_request(self, req_id):
        return self._h.wait_request(int(req_id))

    def pending(self):
        return self._h.pending()

    def get_block_size(self):
        return self._h.get_block_size()

    def get_queue_depth(self):
        return self._h.get_queue_depth()

    def get_thread_count(self):
        return self._h.get_thread_count()

    @staticmethod
    def new_cpu_locked_tensor(num_elem, example_tensor):
        pin = torch.cuda.is_available()
        return torch.empty(int(num_elem), dtype=example_tensor.dtype, pin_memory=pin)

    @staticmethod
    def free_cpu_locked_tensor(t):
        del t


def aio_handle(*args, **kw):
    return AsyncIOHandle(*args, **kw)
