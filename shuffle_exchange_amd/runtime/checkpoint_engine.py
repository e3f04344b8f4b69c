"""Checkpoint engines (parity: reference runtime/checkpoint_engine/torch_checkpoint_engine.py:15,
decoupled_checkpoint_engine.py:68, fast_checkpoint_engine.py:16).

* ``TorchCheckpointEngine``: synchronous ``torch.save``.
* ``FastCheckpointEngine``: ``torch.save`` streamed through ``io.FastFileWriter`` (pinned double
  buffer -> C++ AIO engine, O_DIRECT); reference fast_checkpoint_engine.py:16.
* ``AsyncCheckpointEngine`` (the decoupled engine): tensors are snapshotted to pinned host memory on
  a side HIP stream (no GPU stall beyond the D2H copy), then a background thread serialises them;
  ``commit()`` waits. Training continues while the file is written.
Everything is loaded with ``torch.load(weights_only=True)``: checkpoints contain only tensors and
plain containers.
"""
import os
import threading

import torch

from ..accelerator import get_accelerator


class CheckpointEngine:
    def create(self, tag):
        pass

    def makedirs(self, path, exist_ok=False):
        os.makedirs(path, exist_ok=exist_ok)

    def save(self, state_dict, path):
        raise NotImplementedError

    def load(self, path, map_location=None):
        return torch.load(path, map_location=map_location, weights_only=True)

    def commit(self, tag):
        return True

    def wait(self):
        pass


class TorchCheckpointEngine(CheckpointEngine):
    def save(self, state_dict, path):
        tmp = path + ".tmp"
        torch.save(state_dict, tmp)
        os.replace(tmp, path)


def _to_host(obj, stream):
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            h = torch.empty(obj.shape, dtype=obj.dtype, pin_memory=True)
            with torch.cuda.stream(stream):
                h.copy_(obj, non_blocking=True)
            return h
        return obj.clone()
    if isinstance(obj, dict):
        return type(obj)((k, _to_host(v, stream)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v, stream) for v in obj)
    return obj


class AsyncCheckpointEngine(CheckpointEngine):
    def __init__(self):
        self._threads = []
        self._errors = []
        acc = get_accelerator()
        self.stream = acc.named_stream("ckpt_d2h") if acc.gpu else None

    def save(self, state_dict, path):
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream())
        snap = _to_host(state_dict, self.stream)
        ev = None
        if self.stream is not None:
            ev = torch.cuda.Event()
            ev.record(self.stream)

        def run():
            try:
                if ev is not None:
                    ev.synchronize()
                tmp = path + ".tmp"
                torch.save(snap, tmp)
                os.replace(tmp, path)
            except Exception as e:  # pragma: no cover
                self._errors.append(e)

        t = threading.Thread(target=run, daemon=True)
        t.start()
        self._threads.append(t)

    def wait(self):
        for t in self._threads:
            t.join()
        self._threads = []
        if self._errors:
            e = self._errors[0]
            self._errors = []
            raise e

    def commit(self, tag):
        self.wait()
        return True


class FastCheckpointEngine(CheckpointEngine):
    def __init__(self, config_params=None, buffer_size=64 << 20):
        from ..io import FastFileWriterConfig
        self.cfg = FastFileWriterConfig(buffer_size=buffer_size)

    def save(self, state_dict, path):
        from ..io import FastFileWriter
        tmp = path + ".tmp"
        w = FastFileWriter(tmp, self.cfg)
        torch.save(state_dict, w)
        w.close()
        os.replace(tmp, path)


DecoupledCheckpointEngine = AsyncCheckpointEngine
