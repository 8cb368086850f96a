"""OnDevice context (reference `utils/init_on_device.py:12`): construct modules directly on a device (or on `meta`
for zero-memory shape-only construction) and in a target dtype."""
import torch


class OnDevice:

    _orig_torch_empty = None

    def __init__(self, dtype=None, device="meta", enabled=True):
        self.dtype = dtype
        self.device = torch.device(device)
        self.enabled = enabled
        self._ctx = None
        self._prev_dtype = None

    def __enter__(self):
        if not self.enabled:
            return self
        self._ctx = torch.device(self.device)
        self._ctx.__enter__()
        if self.dtype is not None:
            self._prev_dtype = torch.get_default_dtype()
            torch.set_default_dtype(self.dtype)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        if self._prev_dtype is not None:
            torch.set_default_dtype(self._prev_dtype)
        self._ctx.__exit__(*exc)
        return False
