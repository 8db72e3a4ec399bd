"""``OnDevice``: build a model directly on a device or as meta tensors (reference utils/init_on_device.py :12).

``with OnDevice(dtype=torch.bfloat16, device="meta"): model = Model()`` allocates nothing; ``device="cuda"``
allocates parameters straight in HBM in the target dtype (no host staging of a 70B model). Implemented with
torch's device context plus a default-dtype switch, so every tensor constructor (nn.Linear's ``torch.empty``,
``torch.zeros`` ...) lands on the target device in the target dtype.
"""
import torch


class OnDevice:

    def __init__(self, dtype, device="meta", enabled=True):
        self.dtype = dtype
        self.enabled = enabled
        self.device = torch.device(device) if isinstance(device, str) else device
        if self.device.type == "cuda" and self.device.index is None and torch.cuda.is_available():
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._prev_default = None
        self._dev_ctx = None

    def __enter__(self):
        if not self.enabled:
            return self
        self._prev_default = torch.get_default_dtype()
        self._dev_ctx = torch.device(self.device)
        self._dev_ctx.__enter__()
        if self.dtype is not None and self.dtype.is_floating_point:
            torch.set_default_dtype(self.dtype)
        return self

    def __exit__(self, exc_type, exc_value, traceback):
        if not self.enabled:
            return False
        torch.set_default_dtype(self._prev_default)
        self._dev_ctx.__exit__(exc_type, exc_value, traceback)
        return False
