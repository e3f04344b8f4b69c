"""``OnDevice``: construct modules directly on a device (or as meta tensors) in a given dtype.

Parity: reference utils/init_on_device.py:12 ``OnDevice(dtype, device="meta", enabled=True)``. The
reference monkey-patches torch.empty/zeros/ones/full; PyTorch 2.x offers the same through the
device context manager plus the default dtype, which also covers nn.Module parameter factories.
On MI355X, ``device=f"cuda:{local_rank}"`` builds an 8B model straight into HBM (no host copy);
``device="meta"`` builds a shape-only skeleton for checkpoint-driven materialisation
(``module.to_empty(device=...)``).
"""
import torch


class OnDevice:
    def __init__(self, dtype, device="meta", enabled=True):
        self.dtype, self.device, self.enabled = dtype, device, enabled

    def __enter__(self):
        if not self.enabled:
            return self
        self._prev = torch.get_default_dtype()
        if self.dtype is not None and self.dtype.is_floating_point:
            torch.set_default_dtype(self.dtype)
        self._ctx = torch.device(self.device)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        self._ctx.__exit__(*exc)
        torch.set_default_dtype(self._prev)
        return False
