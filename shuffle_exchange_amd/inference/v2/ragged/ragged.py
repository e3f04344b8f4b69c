"""Ragged-batch state for the FastGen-style engine: block allocator, blocked KV cache, sequence
descriptors, state manager and the per-forward ragged batch metadata.

Parity: reference inference/v2/ragged/ -- ``BlockedAllocator`` (blocked_allocator.py:11),
``BlockedKVCache`` (kv_cache.py:40), ``DSSequenceDescriptor`` (sequence_descriptor.py:59),
``DSStateManager`` (ragged_manager.py:19), ``RaggedBatchWrapper`` (ragged_wrapper.py:31).

MI355X-first sizing: the KV cache is one allocation per model ([layers, blocks, 2, nkv, bs, D]),
sized from a fraction of the free HBM (288 GB per GPU => hundreds of thousands of tokens of
Llama-3-8B KV at bf16); the batch metadata is built in pinned host buffers and crosses to the GPU
in one copy per dtype.
"""
from dataclasses import dataclass, field
from typing import List

import torch


class BlockedAllocator:
    """Free-list allocator of KV block ids (host side, O(1) alloc/free)."""

    def __init__(self, num_blocks):
        if num_blocks < 1:
            raise ValueError("num_blocks must be positive")
        self._num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))
        self._used = [False] * num_blocks

    @property
    def free_blocks(self):
        return len(self._free)

    @property
    def num_blocks(self):
        return self._num_blocks

    def allocate(self, num_blocks):
        if num_blocks > len(self._free):
            raise ValueError(f"not enough free KV blocks ({num_blocks} > {len(self._free)})")
        out = [self._free.pop() for _ in range(num_blocks)]
        for b in out:
            self._used[b] = True
        return torch.tensor(out, dtype=torch.int32)

    def free(self, blocks):
        for b in (blocks.tolist() if torch.is_tensor(blocks) else list(blocks)):
            if not (0 <= b < self._num_blocks) or not self._used[b]:
                raise ValueError(f"invalid free of block {b}")
            self._used[b] = False
            self._free.append(b)


class BlockedKVCache:
    def __init__(self, num_layers, num_blocks, block_size, n_kv_heads, head_dim, dtype=torch.bfloat16, device=None):
        self.num_layers, self.num_blocks, self.block_size = num_layers, num_blocks, block_size
        self.n_kv_heads, self.head_dim = n_kv_heads, head_dim
        self.cache = torch.zeros(num_layers, num_blocks, 2, n_kv_heads, block_size, head_dim, dtype=dtype,
                                 device=device)
        self.allocator = BlockedAllocator(num_blocks)

    @staticmethod
    def blocks_for_budget(budget_bytes, num_layers, block_size, n_kv_heads, head_dim, dtype=torch.bfloat16):
        per_block = num_layers * 2 * n_kv_heads * block_size * head_dim * torch.tensor([], dtype=dtype).element_size()
        return max(1, int(budget_bytes // per_block))

    def layer(self, i):
        return self.cache[i]

    def reserve(self, n):
        return self.allocator.allocate(n)

    def free(self, blocks):
        self.allocator.free(blocks)

    @property
    def free_blocks(self):
        return self.allocator.free_blocks


@dataclass
class DSSequenceDescriptor:
    uid: int
    max_blocks: int
    seen_tokens: int = 0
    in_flight_tokens: int = 0
    blocks: List[int] = field(default_factory=list)

    @property
    def cur_allocated_blocks(self):
        return len(self.blocks)

    def blocks_needed(self, new_tokens, block_size):
        total = self.seen_tokens + new_tokens
        return max(0, (total + block_size - 1) // block_size - len(self.blocks))

    def pre_forward(self, n):
        self.in_flight_tokens = n

    def post_forward(self):
        self.seen_tokens += self.in_flight_tokens
        self.in_flight_tokens = 0


class DSStateManager:
    def __init__(self, kv_cache: BlockedKVCache, max_tracked_sequences=2048, max_blocks_per_sequence=None):
        self.kv = kv_cache
        self.max_tracked = max_tracked_sequences
        self.max_blocks_per_seq = max_blocks_per_sequence or kv_cache.num_blocks
        self.seqs = {}

    @property
    def n_tracked_sequences(self):
        return len(self.seqs)

    @property
    def free_blocks(self):
        return self.kv.free_blocks

    def get_sequence(self, uid):
        return self.seqs.get(uid)

    def get_or_create_sequence(self, uid):
        s = self.seqs.get(uid)
        if s is None:
            if len(self.seqs) >= self.max_tracked:
                raise RuntimeError(f"tracking limit of {self.max_tracked} sequences reached")
            s = DSSequenceDescriptor(uid, self.max_blocks_per_seq)
            self.seqs[uid] = s
        return s

    def allocate_blocks(self, seq, n_new_tokens):
        need = seq.blocks_needed(n_new_tokens, self.kv.block_size)
        if need:
            if len(seq.blocks) + need > seq.max_blocks:
                raise RuntimeError(f"sequence {seq.uid} exceeds {seq.max_blocks} KV blocks")
            seq.blocks.extend(self.kv.reserve(need).tolist())

    def flush_sequence(self, uid):
        s = self.seqs.pop(uid, None)
        if s is not None and s.blocks:
            self.kv.free(s.blocks)


class RaggedBatch:
    """Device metadata of one forward over a ragged set of sequences (all int tensors on device).

    input_ids [T]; positions [T] (absolute); slots [T] (cache slot of every new token);
    q_start / q_len / kv_len [S] int32; block_table [S, max_blocks] int32; last_idx [S] int64.
    Host copies of the small per-sequence ints are kept for scheduling decisions.
    """

    def __init__(self, seqs, tokens, block_size, device):
        S = len(seqs)
        lens = [int(t.numel()) for t in tokens]
        T = sum(lens)
        maxb = max(1, max(len(s.blocks) for s in seqs))
        i64 = torch.empty(3 * T + S, dtype=torch.int64, pin_memory=torch.cuda.is_available() and device.type == "cuda")
        i32 = torch.zeros(3 * S + S * maxb, dtype=torch.int32,
                          pin_memory=torch.cuda.is_available() and device.type == "cuda")
        ids, pos, slots, last = i64[:T], i64[T:2 * T], i64[2 * T:3 * T], i64[3 * T:]
        qs, ql, kl = i32[:S], i32[S:2 * S], i32[2 * S:3 * S]
        bt = i32[3 * S:].view(S, maxb)
        t = 0
        self.host_q_len, self.host_kv_len, self.host_seen = [], [], []
        for i, (s, tk) in enumerate(zip(seqs, tokens)):
            n = lens[i]
            ids[t:t + n] = tk.to(torch.int64)
            p = torch.arange(s.seen_tokens, s.seen_tokens + n, dtype=torch.int64)
            pos[t:t + n] = p
            blk = torch.tensor(s.blocks, dtype=torch.int64)
            slots[t:t + n] = blk[p // block_size] * block_size + p % block_size
            qs[i], ql[i], kl[i] = t, n, s.seen_tokens + n
            bt[i, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
            last[i] = t + n - 1
            self.host_q_len.append(n)
            self.host_kv_len.append(s.seen_tokens + n)
            self.host_seen.append(s.seen_tokens)
            t += n
        d64 = i64.to(device, non_blocking=True)
        d32 = i32.to(device, non_blocking=True)
        self.input_ids, self.positions, self.slots, self.last_idx = d64[:T], d64[T:2 * T], d64[2 * T:3 * T], d64[3 * T:]
        self.q_start, self.q_len, self.kv_len = d32[:S], d32[S:2 * S], d32[2 * S:3 * S]
        self.block_table = d32[3 * S:].view(S, maxb)
        self.num_tokens, self.num_seqs = T, S
        self.max_kv_len = max(self.host_kv_len) if S else 0
        self.host_q_start = [sum(lens[:i]) for i in range(S)]
