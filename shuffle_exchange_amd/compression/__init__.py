"""Compression (reference compression/)."""
from .compress import LinearLayer_Compress, compression_scheduler, init_compression, redundancy_clean  # noqa: F401
