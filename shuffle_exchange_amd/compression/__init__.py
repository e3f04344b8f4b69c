"""Compression (reference compression/)."""
from .compress import (BNLayer_Compress, Conv2dLayer_Compress, Embedding_Compress, LinearLayer_Compress,  # noqa: F401
                       compression_scheduler, init_compression, redundancy_clean)
