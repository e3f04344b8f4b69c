from .ragged import (BlockedAllocator, BlockedKVCache, DSSequenceDescriptor, DSStateManager,  # noqa: F401
                     RaggedBatch)
