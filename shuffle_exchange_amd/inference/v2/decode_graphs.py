"""HIP-graph replay of decode steps for the ragged engine.

A decode step of a dense model (every sequence adds ONE token) is launch-bound at serving batch
sizes: Llama-3-8B issues ~10 kernels per layer (norm, QKV GEMM, RoPE, KV append, paged attention
(+ split merge), O GEMM, norm, gate/up GEMM, SwiGLU, down GEMM), i.e. ~330 launches per token,
while the HBM time of the step is ~2 ms. The reference captures CUDA graphs only in its v1 engine
(inference/engine.py ``_create_cuda_graph``); here the v2 engine captures its decode steps:

* graphs are keyed by (sequence bucket, KV-length bucket), both powers of two, captured lazily on
  first use and sharing one memory pool;
* all per-step metadata (token ids, positions, cache slots, block tables, lengths) lives in static
  device buffers refreshed by one pinned H2D copy per dtype before ``replay()``;
* padding sequences point at a reserved scratch KV block (q_len = kv_len = 1), so every row the
  graph computes is well defined and no real cache slot is touched;
* the paged-attention grid is fixed per graph by the KV bucket (splits of >= 256 keys, workgroups
  past a sequence's length exit at once).

MoE models (data-dependent expert counts) and sliding windows narrower than the KV bucket run
eagerly.
"""
import torch

MIN_KV_BUCKET = 256


def _pow2_at_least(n, lo=1):
    b = lo
    while b < n:
        b *= 2
    return b


class _StaticBatch:
    """RaggedBatch protocol (see ragged.py) over fixed-shape device buffers."""

    def __init__(self, S, max_blocks, kv_bucket, device):
        self.num_tokens = self.num_seqs = S
        self.max_blocks = max_blocks
        self.max_kv_len = kv_bucket
        self.d64 = torch.zeros(4 * S, dtype=torch.int64, device=device)
        self.d32 = torch.zeros(3 * S + S * max_blocks, dtype=torch.int32, device=device)
        self.h64 = torch.zeros(4 * S, dtype=torch.int64, pin_memory=True)
        self.h32 = torch.zeros(3 * S + S * max_blocks, dtype=torch.int32, pin_memory=True)
        self.input_ids, self.positions, self.slots, self.last_idx = self.d64.view(4, S).unbind(0)
        self.q_start, self.q_len, self.kv_len = self.d32[:3 * S].view(3, S).unbind(0)
        self.block_table = self.d32[3 * S:].view(S, max_blocks)
        # host views read by the attention dispatch: no pure prefill, every row one query token
        self.host_seen = [1] * S
        self.host_q_len = [1] * S
        self.host_q_start = list(range(S))
        self.host_kv_len = [kv_bucket] * S
        self.copied = None  # event: last H2D copy out of the pinned buffers


class DecodeGraphRunner:
    def __init__(self, model, kv_cache, max_seqs=256, max_context=131072):
        self.model, self.kv = model, kv_cache
        self.max_seqs = max_seqs
        self.max_context = max_context
        self.bs = kv_cache.block_size
        self.scratch_block = int(kv_cache.reserve(1)[0])
        self._graphs = {}
        self._pool = None
        self.replays = 0

    # ------------------------------------------------------------------------------ eligibility
    def eligible(self, seqs, lens):
        if not lens or any(n != 1 for n in lens) or len(seqs) > self.max_seqs:
            return False
        kv_max = max(s.seen_tokens + 1 for s in seqs)
        if kv_max > self.max_context:
            return False
        window = getattr(getattr(self.model, "spec", None), "sliding_window", None)
        if window is not None and self._kv_bucket(kv_max) > window:
            return False
        return True

    def _kv_bucket(self, kv_max):
        return max(_pow2_at_least(kv_max, MIN_KV_BUCKET), self.bs)

    # ------------------------------------------------------------------------------------- run
    def run(self, seqs, tokens):
        S_real = len(seqs)
        S = _pow2_at_least(S_real)
        kvb = self._kv_bucket(max(s.seen_tokens + 1 for s in seqs))
        key = (S, kvb)
        entry = self._graphs.get(key)
        sb = entry[1] if entry is not None else _StaticBatch(S, (kvb + self.bs - 1) // self.bs, kvb,
                                                              self.model.device)
        self._fill(sb, seqs, tokens)
        if entry is None:
            entry = self._capture(sb)
            self._graphs[key] = entry
        graph, _, out = entry
        graph.replay()
        self.replays += 1
        return out[:S_real].clone()

    def _fill(self, sb, seqs, tokens):
        if sb.copied is not None:
            sb.copied.synchronize()  # the previous step's copy has left the pinned buffers
        S, mb, bs = sb.num_seqs, sb.max_blocks, self.bs
        h64, h32 = sb.h64.view(4, S), sb.h32
        ids, pos, slots, last = h64.unbind(0)
        qs, ql, kl = h32[:3 * S].view(3, S).unbind(0)
        bt = h32[3 * S:].view(S, mb)
        scratch_slot = self.scratch_block * bs
        ids.zero_()
        pos.zero_()
        slots.fill_(scratch_slot)
        last.copy_(torch.arange(S))
        qs.copy_(torch.arange(S, dtype=torch.int32))
        ql.fill_(1)
        kl.fill_(1)
        bt.fill_(self.scratch_block)
        for i, (s, t) in enumerate(zip(seqs, tokens)):
            p = s.seen_tokens
            ids[i] = int(t.reshape(-1)[0])
            pos[i] = p
            slots[i] = s.blocks[p // bs] * bs + p % bs
            kl[i] = p + 1
            nb = len(s.blocks)
            bt[i, :nb] = torch.tensor(s.blocks, dtype=torch.int32)
        sb.d64.copy_(sb.h64, non_blocking=True)
        sb.d32.copy_(sb.h32, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        sb.copied = ev

    def _capture(self, sb):
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), torch.no_grad():
            self.model.forward(sb, self.kv)  # warm-up: lazy inits, hipBLASLt heuristics; same KV writes as replay
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self._pool), torch.no_grad():
            out = self.model.forward(sb, self.kv)
        return graph, sb, out

    @property
    def num_graphs(self):
        return len(self._graphs)
