"""Trace ranges (reference utils/nvtx.py:12 ``instrument_w_nvtx``).

On ROCm ``torch.cuda.nvtx`` emits roctx ranges, which ``rocprofv3 --marker-trace`` records next to
the kernel trace. Ranges are only pushed when ``SXE_ROCTX=1`` (the accelerator's switch): a
push/pop pair costs microseconds of host time, which matters in launch-bound loops."""
import functools
import os


def instrument_w_nvtx(func):
    """Decorator: wrap ``func`` in a trace range named after it."""
    if os.environ.get("SXE_ROCTX", "0") != "1":
        return func
    from ..accelerator import get_accelerator

    @functools.wraps(func)
    def wrapped(*args, **kwargs):
        acc = get_accelerator()
        acc.range_push(func.__qualname__)
        try:
            return func(*args, **kwargs)
        finally:
            acc.range_pop()

    return wrapped
