"""Point-to-point activation / gradient transfer between adjacent pipeline stages.

Parity: reference runtime/pipe/p2p.py (``send`` :46, ``recv`` :67, ``_is_valid_send_recv`` and
``init_process_groups``) plus the metadata handshake of runtime/pipe/engine.py ``_send_tensor_meta``
:900 / ``_recv_tensor_meta`` :943.

MI355X: every adjacent pair of GPUs on a node has a direct xGMI link, so the transfer is a plain
RCCL send/recv on the global communicator (no 2-rank broadcast groups as the reference's fallback
uses). Sends are non-blocking (``isend``) and kept alive until the step ends; only receives block.
Metadata (count, dtype, shape, requires_grad per tensor) travels in one small int64 message before
the first payload of every batch, so a stage never needs to know its neighbour's shapes.
"""
import torch

from ... import comm as dist

_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool, torch.uint8,
           torch.float64, torch.int16, torch.int8]
_CODE = {d: i for i, d in enumerate(_DTYPES)}
_MAX_META = 64


def _as_tuple(x):
    return x if isinstance(x, (tuple, list)) else (x,)


class P2PChannel:
    """Adjacent-stage transfers for one pipeline engine (one per rank)."""

    def __init__(self, grid, device):
        self.grid = grid
        self.device = device
        self.pending = []  # outstanding isend work handles (+ tensors kept alive)

    def _peer(self, stage_id):
        return self.grid.stage_to_global(stage_id)

    # ---------------------------------------------------------------------------- metadata
    def send_meta(self, tensors, dst_stage):
        tensors = _as_tuple(tensors)
        meta = [len(tensors)]
        for t in tensors:
            meta += [_CODE[t.dtype], int(t.requires_grad), t.dim(), *t.shape]
        assert len(meta) <= _MAX_META, "activation metadata too large"
        buf = torch.zeros(_MAX_META, dtype=torch.int64, device=self.device)
        buf[:len(meta)] = torch.tensor(meta, dtype=torch.int64)
        self._isend(buf, dst_stage)

    def recv_meta(self, src_stage):
        buf = torch.empty(_MAX_META, dtype=torch.int64, device=self.device)
        dist.recv(buf, src=self._peer(src_stage))
        m = buf.tolist()
        n, i, out = m[0], 1, []
        for _ in range(n):
            code, rg, nd = m[i], m[i + 1], m[i + 2]
            shape = tuple(m[i + 3:i + 3 + nd])
            out.append((_DTYPES[code], bool(rg), shape))
            i += 3 + nd
        return out

    # ---------------------------------------------------------------------------- payload
    def _isend(self, t, dst_stage):
        work = dist.isend(t.contiguous(), dst=self._peer(dst_stage))
        self.pending.append((work, t))

    def send(self, tensors, dst_stage):
        for t in _as_tuple(tensors):
            self._isend(t.detach(), dst_stage)

    def recv(self, meta, src_stage):
        out = []
        for dtype, rg, shape in meta:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            dist.recv(t, src=self._peer(src_stage))
            out.append(t)
        return out

    def wait_sends(self):
        for work, _ in self.pending:
            if work is not None:
                work.wait()
        self.pending = []
