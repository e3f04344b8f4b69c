"""Ulysses sequence parallelism (parity: reference sequence/layer.py, runtime/sequence_parallel/) and ring
attention / context parallelism (new: sequence/ring_attention.py)."""
from .data import UlyssesSPDataLoaderAdapter, shard_batch_for_sp  # noqa: F401
from .layer import DistributedAttention, head_to_seq, seq_to_head, ulysses_qkv_attention  # noqa: F401
from .tiled import (SequenceTiledCompute, TiledMLP, UlyssesSPAttentionHF, register_with_transformers,  # noqa: F401
                    sequence_tiled_compute, tiled_fused_logits_loss, vocab_sequence_parallel_cross_entropy)
from .ring_attention import ring_attention, ring_qkv_attention, zigzag_shard  # noqa: F401,E402
