"""NVMe / async-I/O benchmarking and tuning (reference deepspeed/nvme: ds_io, ds_nvme_tune)."""
from .io_bench import io_benchmark, parse_size, sweep, main  # noqa: F401
