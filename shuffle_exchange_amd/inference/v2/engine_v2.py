"""FastGen-style continuous-batching inference engine.

Parity: reference inference/v2/engine_v2.py -- ``InferenceEngineV2`` :30 with ``put`` :107-156
(ragged batch of new tokens for many sequences -> last-token logits), ``query`` :158 (how many
tokens / KV blocks a sequence may still take), ``can_schedule`` :184, ``flush`` :242,
``serialize``; config ``RaggedInferenceEngineConfig`` (state_manager: max_tracked_sequences,
max_ragged_batch_size, max_ragged_sequence_count, memory_config) and ``build_hf_engine``
(engine_factory.py) -- here ``build_engine(model, config)`` since models are this framework's own
(no hub access).

Each ``put`` is one forward over the concatenated new tokens of all listed sequences: prompts
(prefill, any length), continuations (decode) and chunked prefills mix freely. KV blocks are
allocated on demand from the blocked cache and returned on ``flush``.
"""
import math
from dataclasses import dataclass, field
from enum import Enum
from typing import Optional

import torch

from .ragged.ragged import BlockedKVCache, DSStateManager, RaggedBatch


class SchedulingResult(Enum):
    Success = 0
    EngineSequenceLimitExceeded = 1
    BatchSequenceLimitExceeded = 2
    BatchTokenLimitExceeded = 3
    KVCacheLimitExceeded = 4
    SequenceTokenLimitExceeded = 5


class SchedulingError(RuntimeError):
    def __init__(self, result):
        super().__init__(f"batch scheduling failed: {result.name}")
        self.result = result


@dataclass
class MemoryConfig:
    mode: str = "reserve"          # "reserve": leave `size` bytes free; "allocate": use `size` bytes
    size: int = 16 * 2**30
    fraction: Optional[float] = None  # alternative: fraction of the currently free device memory


@dataclass
class StateManagerConfig:
    max_tracked_sequences: int = 2048
    max_ragged_batch_size: int = 8192
    max_ragged_sequence_count: int = 512
    max_context: int = 131072
    memory_config: MemoryConfig = field(default_factory=MemoryConfig)
    offload: bool = False


@dataclass
class RaggedInferenceEngineConfig:
    state_manager: StateManagerConfig = field(default_factory=StateManagerConfig)
    kv_block_size: int = 64
    num_kv_blocks: Optional[int] = None
    tensor_parallel: dict = field(default_factory=lambda: {"tp_size": 1})
    decode_graphs: bool = True  # replay pure-decode steps from captured HIP graphs (decode_graphs.py)
    weight_quant: Optional[str] = None  # "fp8" (W8A16) | "fp6" / "wf6af16" (FP6-LLM) | "fp4": weight-only decode GEMMs
    implementations: Optional[dict] = None  # pin registry implementations by interface (modules/registry.py)


_TP_GROUPS = {}


def _tp_group(tp):
    """Consecutive blocks of `tp` ranks (the ranks of one node share one xGMI mesh); created once
    per (tp, world) so build_hf_engine and the engine share it."""
    from ... import comm as dist
    assert dist.is_initialized(), "tensor_parallel.tp_size > 1 needs torch.distributed"
    world, me = dist.get_world_size(), dist.get_rank()
    assert world % tp == 0, f"world size {world} must be a multiple of tp_size {tp}"
    if tp == world:
        return None  # the world group
    key = (tp, world, id(dist.get_world_group()) if hasattr(dist, "get_world_group") else 0)
    if key in _TP_GROUPS:
        return _TP_GROUPS[key]
    mine = None
    for i in range(0, world, tp):
        g = dist.new_group(list(range(i, i + tp)))  # every rank creates every group
        if i <= me < i + tp:
            mine = g
    _TP_GROUPS[key] = mine
    return mine


class InferenceEngineV2:
    def __init__(self, model, config: RaggedInferenceEngineConfig = None):
        from .model_implementations import ragged_model_for
        self._config = config or RaggedInferenceEngineConfig()
        tp = int((self._config.tensor_parallel or {}).get("tp_size", 1))
        self._tp = tp
        self._tp_group = _tp_group(tp) if tp > 1 else None
        self._model = ragged_model_for(model, weight_quant=self._config.weight_quant, tp_group=self._tp_group,
                                       tp_size=tp, pins=self._config.implementations)
        sm = self._config.state_manager
        dev = self._model.device
        bs = self._config.kv_block_size
        nblocks = self._config.num_kv_blocks or self._size_cache(dev, bs)
        self._kv = BlockedKVCache(self._model.num_layers, nblocks, bs, self._model.nkv, self._model.head_dim,
                                  dtype=self._model.dtype, device=dev)
        max_blocks_seq = math.ceil(sm.max_context / bs)
        self._state = DSStateManager(self._kv, sm.max_tracked_sequences, max_blocks_seq)
        self._decode_graphs = None

    def _size_cache(self, dev, bs):
        m = self._model
        mc = self._config.state_manager.memory_config
        if dev.type != "cuda":
            budget = 64 * 2**20
        else:
            free, _ = torch.cuda.mem_get_info(dev)
            if mc.fraction is not None:
                budget = int(free * mc.fraction)
            elif mc.mode == "allocate":
                budget = mc.size
            else:
                budget = max(0, free - mc.size)
        return BlockedKVCache.blocks_for_budget(budget, m.num_layers, bs, m.nkv, m.head_dim, m.dtype)

    # ------------------------------------------------------------------------------------ API
    @property
    def free_blocks(self):
        return self._state.free_blocks

    @property
    def n_kv_blocks(self):
        return self._kv.num_blocks

    @property
    def model(self):
        return self._model

    def put(self, batch_uids, batch_tokens, do_checks=True):
        """Run one forward over the new tokens of every listed sequence; returns [n_seqs, vocab]
        fp32 logits of each sequence's last new token."""
        tokens = [t if torch.is_tensor(t) else torch.tensor(t) for t in batch_tokens]
        tokens = [t.reshape(-1).cpu() for t in tokens]
        if do_checks:
            r = self.can_schedule(batch_uids, [t.numel() for t in tokens])
            if r != SchedulingResult.Success:
                raise SchedulingError(r)
        seqs = []
        for uid, t in zip(batch_uids, tokens):
            s = self._state.get_or_create_sequence(uid)
            self._state.allocate_blocks(s, t.numel())
            s.pre_forward(t.numel())
            seqs.append(s)
        runner = self._decode_runner()
        if runner is not None and runner.eligible(seqs, [t.numel() for t in tokens]):
            logits = runner.run(seqs, tokens)
        else:
            batch = RaggedBatch(seqs, tokens, self._kv.block_size, self._model.device)
            logits = self._model.forward(batch, self._kv)
        for s in seqs:
            s.post_forward()
        return logits

    def _decode_runner(self):
        """HIP-graph decode runner (decode_graphs.py), created on first use: GPU, dense models."""
        if self._decode_graphs is None:
            m = self._model
            dense = not getattr(m, "is_moe", False) and not any(
                "router" in L for L in getattr(m, "w", {}).get("layers", []))
            ok = (self._config.decode_graphs and m.device.type == "cuda" and dense and self._kv.free_blocks > 1
                  and self._tp == 1)  # collectives stay outside graph capture
            if ok:
                from .decode_graphs import DecodeGraphRunner
                sm = self._config.state_manager
                self._decode_graphs = DecodeGraphRunner(m, self._kv, max_seqs=min(256, sm.max_ragged_sequence_count),
                                                        max_context=sm.max_context)
            else:
                self._decode_graphs = False
        return self._decode_graphs or None

    def query(self, uid, max_request_tokens, max_request_blocks):
        """(tokens, blocks) the sequence could take now, bounded by the request and free blocks."""
        bs = self._kv.block_size
        s = self._state.get_sequence(uid)
        seen = s.seen_tokens if s is not None else 0
        have = s.cur_allocated_blocks if s is not None else 0
        free_in_have = have * bs - seen
        blocks = min(max_request_blocks, self._state.free_blocks)
        tokens = min(max_request_tokens, free_in_have + blocks * bs)
        need_blocks = max(0, math.ceil((seen + tokens) / bs) - have)
        return tokens, need_blocks

    def can_schedule(self, uids, lengths):
        sm = self._config.state_manager
        new_seqs = sum(1 for u in uids if self._state.get_sequence(u) is None)
        if self._state.n_tracked_sequences + new_seqs > sm.max_tracked_sequences:
            return SchedulingResult.EngineSequenceLimitExceeded
        if len(uids) > sm.max_ragged_sequence_count:
            return SchedulingResult.BatchSequenceLimitExceeded
        if sum(lengths) > sm.max_ragged_batch_size:
            return SchedulingResult.BatchTokenLimitExceeded
        bs = self._kv.block_size
        need = 0
        for u, n in zip(uids, lengths):
            s = self._state.get_sequence(u)
            seen = s.seen_tokens if s is not None else 0
            have = s.cur_allocated_blocks if s is not None else 0
            if seen + n > sm.max_context:
                return SchedulingResult.SequenceTokenLimitExceeded
            need += max(0, math.ceil((seen + n) / bs) - have)
        if need > self._state.free_blocks:
            return SchedulingResult.KVCacheLimitExceeded
        return SchedulingResult.Success

    def flush(self, uid):
        self._state.flush_sequence(uid)

    def get_remaining_block_capacity(self, uid):
        s = self._state.get_sequence(uid)
        if s is None:
            return 0
        return s.cur_allocated_blocks * self._kv.block_size - s.seen_tokens

    def serialize(self, save_path):
        """Write this rank's model (weights as served: TP shard, quantized form) plus the metadata
        ``build_engine_from_ds_checkpoint`` rebuilds it from (reference engine_v2.py:251;
        serialization.py). Every tensor-parallel rank calls it."""
        from .serialization import serialize_engine
        return serialize_engine(self, save_path)

    # ----------------------------------------------------------------------------- generation
    @torch.no_grad()
    def generate(self, prompts, max_new_tokens=32, temperature=0.0, top_k=0, eos_token_id=None, seed=None):
        """Continuous-batching generation for a list of prompts (token id lists / tensors).
        Greedy when temperature == 0. Returns the generated ids per prompt."""
        gen = torch.Generator(device="cpu")
        if seed is not None:
            gen.manual_seed(seed)
        base = 1 << 40
        uids = [base + i for i in range(len(prompts))]
        outs = [[] for _ in prompts]
        live = list(range(len(prompts)))
        step_tokens = [torch.as_tensor(p).reshape(-1) for p in prompts]
        try:
            while live:
                logits = self.put([uids[i] for i in live], [step_tokens[i] for i in live])
                nxt = _sample(logits, temperature, top_k, gen)
                new_live = []
                for j, i in enumerate(live):
                    tok = int(nxt[j])
                    outs[i].append(tok)
                    step_tokens[i] = torch.tensor([tok])
                    if len(outs[i]) < max_new_tokens and (eos_token_id is None or tok != eos_token_id):
                        new_live.append(i)
                live = new_live
        finally:
            for u in uids:
                self.flush(u)
        return outs


def _sample(logits, temperature, top_k, gen):
    logits = logits.float().cpu()
    if temperature <= 0:
        return logits.argmax(-1)
    logits = logits / temperature
    if top_k and top_k > 0:
        v, _ = logits.topk(top_k, dim=-1)
        logits = logits.masked_fill(logits < v[:, -1:], float("-inf"))
    return torch.multinomial(torch.softmax(logits, -1), 1, generator=gen).squeeze(-1)


def build_engine(model, engine_config=None):
    """Serve a framework model (LlamaForCausalLM / MixtralForCausalLM) with the ragged engine
    (reference engine_factory.build_hf_engine)."""
    model.eval()
    return InferenceEngineV2(model, engine_config)
