"""Ulysses sequence parallelism (parity: reference sequence/layer.py, runtime/sequence_parallel/)."""
from .data import UlyssesSPDataLoaderAdapter, shard_batch_for_sp  # noqa: F401
from .layer import DistributedAttention, head_to_seq, seq_to_head, ulysses_qkv_attention  # noqa: F401
